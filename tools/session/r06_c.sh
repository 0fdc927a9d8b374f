#!/bin/bash
# round 6 session C: k_levels_seg v2 (table walk + lane buffers) — level parity tests, phase stamps, cfg2 alone
cd "$GRAFT_REPO_ROOT"
B="python bench.py --no-cpu-baseline --no-e2e --steps 20 --warmup 3"
tools/gpu_steps.sh \
  "300 tests python -u -m pytest tests/test_levels_seg.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "200 diag python tools/diag.py cfg2" \
  "200 b_v2_one env PQ_ONE_STREAM=1 $B" \
  "200 b_v2 $B"
