#!/bin/bash
# round 6 closing evidence, part 1 (build of this commit): GPU suite, smoke, the driver's default line,
# every config's line, full-size verification of cfg2 / cfg3 / cfg4 and the sampled cfg5 check
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
  "300 v2 $B --config cfg2 --verify" \
  "300 v3 $B --config cfg3 --verify" \
  "400 v4 $B --config cfg4 --verify"
