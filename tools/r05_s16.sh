#!/bin/bash
# Round 5 session 16: the whole GPU suite on the current build; cfg2 with the validity bitmaps zeroed
# on the level stream (DELTA-major schedule), its timeline; cfg4.
cd "$(dirname "$0")/.."
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
tools/gpu_steps.sh \
  "600 s16_tests python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 s16_cfg2 $B --config cfg2" \
  "200 s16_tl_cfg2 tools/timeline.sh cfg2" \
  "200 s16_cfg4 $B --config cfg4"
