#!/bin/bash
# Round 5 session 42: level-ahead schedule (PQ_LV_AHEAD): the new back-to-back tests, the GPU suite,
# cfg4 with and without it (alternating), cfg4's timeline and full-size verification.
cd "$(dirname "$0")/.."
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --config cfg4"
tools/gpu_steps.sh \
  "200 s42_nested python -u -m pytest tests/test_nested.py -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "600 s42_gpu_all python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 s42_cfg4 $B" \
  "200 s42_cfg4_off env PQ_LV_AHEAD=0 $B" \
  "200 s42_cfg4_b $B" \
  "200 s42_cfg4_off_b env PQ_LV_AHEAD=0 $B" \
  "200 s42_tl tools/timeline.sh cfg4" \
  "300 s42_verify_cfg4 python -u bench.py --config cfg4 --steps 5 --warmup 2 --verify --no-cpu-baseline --no-e2e"
