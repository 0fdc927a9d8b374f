#!/bin/bash
# Round 5 session 31: cfg2 with double-buffered error keys (the per-decode reset on the level stream,
# none in front of k_values_delta); cfg4 with k_nest_tile counting (no k_nest_pcount), byte-array tile
# bases by look-back now that nothing nested runs beside them, against the pre-pass; full GPU suite.
cd "$(dirname "$0")/.."
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
tools/gpu_steps.sh \
  "400 s31_tests python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 s31_cfg2 $B --config cfg2" \
  "200 s31_cfg4 $B --config cfg4" \
  "200 s31_cfg4_presum1 env PQ_BA_PRESUM=1 $B --config cfg4" \
  "200 s31_cfg2_b $B --config cfg2" \
  "200 s31_cfg4_b $B --config cfg4" \
  "200 s31_tl2 tools/timeline.sh cfg2" \
  "200 s31_tl4 tools/timeline.sh cfg4"
