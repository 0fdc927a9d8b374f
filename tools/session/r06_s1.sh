#!/bin/bash
# Round 6 session 1: the new back-to-back DELTA-major and torn look-back tests, the default bench
# line on this box, the copy-shape calibration, then the whole GPU suite.
cd "$(dirname "$0")/../.."
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
tools/gpu_steps.sh \
  "200 s1_newtests $T tests/test_gpu_parity.py::test_back_to_back_delta_major tests/test_nested.py::test_gpu_lookback_torn_publish -s" \
  "200 s1_bench_cfg2 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --config cfg2" \
  "120 s1_copy_shapes tools/ubench/copy_shapes" \
  "700 s1_gpu_all python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests"
