#!/bin/bash
# round 6 session J: GPU suite + smoke on the committed build, the driver's default bench line, every
# config's bench line, rocprofv3 evidence for cfg2
cd "$GRAFT_REPO_ROOT"
B="python bench.py --no-cpu-baseline --no-e2e --steps 20 --warmup 3"
tools/gpu_steps.sh \
  "700 tests python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" \
  "120 smoke python -c 'import __graft_entry__ as g; g.smoke()'" \
  "300 default python bench.py --gpus 1 --steps 20 --warmup 5" \
  "200 cfg1 $B --config cfg1" \
  "200 cfg3 $B --config cfg3" \
  "300 cfg4 $B --config cfg4" \
  "300 cfg5 $B --config cfg5" \
  "700 prof_cfg2 tools/evidence.sh cfg2"
