#!/bin/bash
# Round 5 session 13: k_levels_seg phase D as one uniform step per iteration (parity, cfg2 bench and
# stamps), phase stamps of the nested kernels on cfg4.
cd "$(dirname "$0")/.."
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
T="python -u -m pytest tests/test_levels_seg.py tests/test_gpu_parity.py tests/test_switches.py tests/test_refwriter.py -m gpu -q -x --timeout 120 --timeout-method thread -rf"
tools/gpu_steps.sh \
  "300 s13_tests $T" \
  "200 s13_cfg2 $B --config cfg2" \
  "200 s13_diag_cfg2 python -u tools/diag.py cfg2" \
  "200 s13_diag_nest python -u tools/diag_nest.py" \
  "200 s13_cfg4 $B --config cfg4"
