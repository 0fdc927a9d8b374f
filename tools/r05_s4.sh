#!/bin/bash
# Round 5 session 4: k_ba_emit pair loads (PA) and non-temporal stores, parity + same-box cfg3 / cfg4.
cd "$(dirname "$0")/.."
L=parquet-go-1_amd/lib
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
T="python -u -m pytest tests/test_ba_classes.py tests/test_gpu_parity.py tests/test_delta_bytearray.py tests/test_plain_bytearray.py tests/test_switches.py -m gpu -q -x --timeout 120 --timeout-method thread -rf"
tools/gpu_steps.sh \
  "300 s4_tests $T" \
  "200 s4_cfg3 $B --config cfg3" \
  "200 s4_cfg3_pa0 env PQGPU_LIB=$L/libpqgpu_pa0.so $B --config cfg3" \
  "200 s4_cfg3_pa0nt0 env PQGPU_LIB=$L/libpqgpu_pa0nt0.so $B --config cfg3" \
  "200 s4_cfg3_pa0nto env PQGPU_LIB=$L/libpqgpu_pa0nto.so $B --config cfg3" \
  "200 s4_cfg3_nto env PQGPU_LIB=$L/libpqgpu_nto.so $B --config cfg3" \
  "200 s4_cfg4 $B --config cfg4" \
  "200 s4_cfg4_pa0nt0 env PQGPU_LIB=$L/libpqgpu_pa0nt0.so $B --config cfg4"
