#!/bin/bash
# Round 5 session 12: class-0 byte-array emit with pair-loaded slots in 16-wave workgroups (PA, 4 rounds
# per wave, no spills) against the default 8-wave emit; parity of the variant, same-box cfg3 / cfg4.
cd "$(dirname "$0")/.."
L=parquet-go-1_amd/lib
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
T="python -u -m pytest tests/test_ba_classes.py tests/test_gpu_parity.py tests/test_switches.py -m gpu -q -x --timeout 120 --timeout-method thread -rf"
tools/gpu_steps.sh \
  "300 s12_tests_pa16 env PQGPU_LIB=$L/libpqgpu_pa16.so $T" \
  "200 s12_cfg3 $B --config cfg3" \
  "200 s12_cfg3_pa16 env PQGPU_LIB=$L/libpqgpu_pa16.so $B --config cfg3" \
  "200 s12_cfg4 $B --config cfg4" \
  "200 s12_cfg4_pa16 env PQGPU_LIB=$L/libpqgpu_pa16.so $B --config cfg4"
tools/gpu_steps.sh "200 s12_diag_cfg2 python -u tools/diag.py cfg2"
