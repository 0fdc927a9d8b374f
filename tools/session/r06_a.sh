#!/bin/bash
# round 6 session A: GPU suite on the committed build, default bench line, copy-shape ubench
cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "600 tests python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "120 smoke python -c 'import __graft_entry__ as g; g.smoke()'" \
  "240 bench python bench.py --steps 20 --warmup 5" \
  "120 copy_shapes tools/ubench/copy_shapes"
