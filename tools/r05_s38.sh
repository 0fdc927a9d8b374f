#!/bin/bash
# Round 5 session 38: k_nest_tcount (one-list-level tiles' counts from the run tables) + k_nest_scan,
# then k_nest_tile with known bases -- against its look-back (PQ_NEST_TCOUNT=0); full GPU suite (the
# nested / struct tests run all three nested modes).
cd "$(dirname "$0")/.."
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
tools/gpu_steps.sh \
  "400 s38_tests python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 s38_cfg4 $B --config cfg4" \
  "200 s38_cfg4_lookback env PQ_NEST_TCOUNT=0 $B --config cfg4" \
  "200 s38_cfg4_b $B --config cfg4" \
  "200 s38_cfg4_lookback_b env PQ_NEST_TCOUNT=0 $B --config cfg4" \
  "300 s38_verify_cfg4 python -u bench.py --config cfg4 --steps 5 --warmup 2 --verify --no-cpu-baseline --no-e2e" \
  "200 s38_tl4 tools/timeline.sh cfg4"
