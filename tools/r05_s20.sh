#!/bin/bash
# Round 5 session 20: DELTA window prefetch without a select into the load registers (the compiler had
# put vmcnt(0) -- every earlier output store -- in front of each window's loads); parity, same-box
# cfg2 / cfg5 against the previous build, stamps.
cd "$(dirname "$0")/.."
L=parquet-go-1_amd/lib
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
T="python -u -m pytest tests/test_gpu_parity.py tests/test_delta_shapes.py tests/test_delta_bytearray.py tests/test_switches.py tests/test_refwriter.py -m gpu -q -x --timeout 120 --timeout-method thread -rf"
tools/gpu_steps.sh \
  "300 s20_tests $T" \
  "200 s20_cfg2 $B --config cfg2" \
  "200 s20_cfg2_base env PQGPU_LIB=$L/libpqgpu_base.so $B --config cfg2" \
  "200 s20_cfg2_b $B --config cfg2" \
  "300 s20_cfg5 $B --config cfg5" \
  "300 s20_cfg5_base env PQGPU_LIB=$L/libpqgpu_base.so $B --config cfg5" \
  "200 s20_diag_cfg2 python -u tools/diag.py cfg2"
