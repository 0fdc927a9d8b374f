#!/bin/bash
# Round check on one GPU: the -m gpu parity suite, then one bench line per config
# (each step under its own time limit; tools/gpu_steps.sh stops at a fault/abort/timeout).
cd "$(dirname "$0")/.."
STEPS=()
[ -z "$SKIP_TESTS" ] && STEPS+=("900 gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf")
for c in ${CONFIGS:-cfg2 cfg1 cfg3 cfg4 cfg5}; do
  STEPS+=("300 bench_$c python -u bench.py --config $c ${BENCH_ARGS:---steps 20 --warmup 3}")
done
exec tools/gpu_steps.sh "${STEPS[@]}"
