#!/bin/bash
# round 6 session AA: after removing the dead compile-time variants (PQ_BA_PA / STORES / NOMASK / NT,
# PQ_NEST_TILES): GPU suite, cfg3 / cfg4 lines
cd "$GRAFT_REPO_ROOT"
B="python bench.py --no-cpu-baseline --no-e2e --steps 20 --warmup 3"
tools/gpu_steps.sh \
  "500 tests python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread" \
  "200 cfg3 $B --config cfg3" \
  "300 cfg4 $B --config cfg4"
tools/gpu_steps.sh \
  "200 ab3 python tools/diag_ablate.py cfg3 0,8192,16384,24576,512,256" \
  "300 ab4 env PQ_ONE_STREAM=1 python tools/diag_ablate.py cfg4 0,8192,16384,24576,512"
