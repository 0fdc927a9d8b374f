#!/bin/bash
# Round 5 session 18: k_snappy with non-temporal long-literal copies (snnt1) and ring flushes (snnt2):
# parity of the variants, same-box cfg5.
cd "$(dirname "$0")/.."
L=parquet-go-1_amd/lib
B="python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --config cfg5"
T="python -u -m pytest tests/test_snappy.py tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -rf"
tools/gpu_steps.sh \
  "300 s18_tests_snnt2 env PQGPU_LIB=$L/libpqgpu_snnt2.so $T" \
  "300 s18_cfg5 $B" \
  "300 s18_cfg5_snnt1 env PQGPU_LIB=$L/libpqgpu_snnt1.so $B" \
  "300 s18_cfg5_snnt2 env PQGPU_LIB=$L/libpqgpu_snnt2.so $B" \
  "300 s18_cfg5_b $B"
