#!/bin/bash
# Round 5 session 19: k_ba_emit pass B with lazy flushes (rounds accumulate in the wave's LDS buffer
# until the next would not fit); parity, same-box cfg3 / cfg4 against the previous build (base).
cd "$(dirname "$0")/.."
L=parquet-go-1_amd/lib
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
T="python -u -m pytest tests/test_ba_classes.py tests/test_gpu_parity.py tests/test_delta_bytearray.py tests/test_plain_bytearray.py tests/test_switches.py tests/test_dict_groups.py -m gpu -q -x --timeout 120 --timeout-method thread -rf"
tools/gpu_steps.sh \
  "300 s19_tests $T" \
  "200 s19_cfg3 $B --config cfg3" \
  "200 s19_cfg3_base env PQGPU_LIB=$L/libpqgpu_base.so $B --config cfg3" \
  "200 s19_cfg4 $B --config cfg4" \
  "200 s19_cfg4_base env PQGPU_LIB=$L/libpqgpu_base.so $B --config cfg4"
