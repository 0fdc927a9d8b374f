#!/bin/bash
# session 2 GPU check: parity tests, then the cfg3 / cfg1 bench lines (each step time-limited)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf \
    > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  tail -30 gpurun_out/gpu_tests.log
  [ $rc -ne 0 ] && exit $rc
fi
for c in cfg3 cfg1; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 3 --verify --no-cpu-baseline \
    > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { cat gpurun_out/bench_$c.err | tail -20; exit 1; }
  cat gpurun_out/bench_$c.json
done
