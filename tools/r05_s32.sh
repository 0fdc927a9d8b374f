#!/bin/bash
# Round 5 session 32: DELTA-major decodes (cfg2) without a per-decode join of the level stream (per-stream
# error keys; k_values_delta resets the next decode's keys): full GPU suite, cfg2 bench and timeline;
# k_nest_tile phase stamps on cfg4 (diagnostic build).
cd "$(dirname "$0")/.."
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
tools/gpu_steps.sh \
  "400 s32_tests python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 s32_cfg2 $B --config cfg2" \
  "200 s32_cfg2_b $B --config cfg2" \
  "200 s32_tl2 tools/timeline.sh cfg2" \
  "200 s32_cfg4 $B --config cfg4" \
  "200 s32_diag_nest python -u tools/diag_nest.py" \
  "200 s32_cfg2_c $B --config cfg2"
