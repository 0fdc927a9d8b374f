#!/bin/bash
# Round 5 session 39: serial schedule with byte-array chunks -- the PLAIN copies after the run scan
# (PQ_COPY_AFTER_SCAN, default) against beside it; the committed defaults' full GPU suite; cfg4 timeline.
cd "$(dirname "$0")/.."
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
tools/gpu_steps.sh \
  "400 s39_tests python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 s39_cfg4 $B --config cfg4" \
  "200 s39_cfg4_beside env PQ_COPY_AFTER_SCAN=0 $B --config cfg4" \
  "200 s39_cfg4_b $B --config cfg4" \
  "200 s39_cfg4_beside_b env PQ_COPY_AFTER_SCAN=0 $B --config cfg4" \
  "200 s39_tl4 tools/timeline.sh cfg4" \
  "200 s39_cfg2 $B --config cfg2" \
  "200 s39_cfg3 $B --config cfg3"
