#!/bin/bash
# Round 5 session 1: parity suite on the default build (stride prelude for level streams), then
# same-box bench comparisons of the experiment variants (tools/variant_lib.sh) and the cfg3 phase split.
cd "$(dirname "$0")/.."
L=parquet-go-1_amd/lib
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
tools/gpu_steps.sh \
  "600 s1_gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "300 s1_tests_badirect env PQGPU_LIB=$L/libpqgpu_badirect.so python -u -m pytest tests/test_ba_classes.py tests/test_gpu_parity.py tests/test_delta_bytearray.py tests/test_plain_bytearray.py -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 s1_cfg4 $B --config cfg4" \
  "200 s1_cfg4_nostride env PQGPU_LIB=$L/libpqgpu_nostride.so $B --config cfg4" \
  "200 s1_cfg3 $B --config cfg3" \
  "200 s1_cfg3_badirect env PQGPU_LIB=$L/libpqgpu_badirect.so $B --config cfg3" \
  "200 s1_cfg3_badirectnt env PQGPU_LIB=$L/libpqgpu_badirectnt.so $B --config cfg3" \
  "200 s1_cfg4_badirect env PQGPU_LIB=$L/libpqgpu_badirect.so $B --config cfg4" \
  "200 s1_cfg2 $B --config cfg2" \
  "200 s1_cfg2_copynt1 env PQGPU_LIB=$L/libpqgpu_copynt1.so $B --config cfg2" \
  "200 s1_cfg2_copynt2 env PQGPU_LIB=$L/libpqgpu_copynt2.so $B --config cfg2" \
  "200 s1_diag_ba python -u tools/diag_ba.py cfg3"
