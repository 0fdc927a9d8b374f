#!/bin/bash
# Round 5 session 45: k_nest_tile's struct-group masks in dynamic LDS (rows for the launch's owned
# groups only: 29.9 -> 21.7 KB per workgroup at R = 1). Nested / struct GPU tests on the new build,
# then cfg4 at 5 (default) / 6 / 7 waves per SIMD (91 VGPRs / 80 + 60 B scratch / 72 + 100 B scratch).
cd "$(dirname "$0")/.."
L=parquet-go-1_amd/lib
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --config cfg4"
tools/gpu_steps.sh \
  "300 s45_tests python -u -m pytest tests/test_nested.py tests/test_struct.py -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 s45_cfg4 $B" \
  "200 s45_cfg4_d6 env PQGPU_LIB=$L/libpqgpu_d6.so $B" \
  "200 s45_cfg4_d7 env PQGPU_LIB=$L/libpqgpu_d7.so $B" \
  "200 s45_cfg4_b $B" \
  "200 s45_cfg4_d6_b env PQGPU_LIB=$L/libpqgpu_d6.so $B" \
  "200 s45_cfg4_d7_b env PQGPU_LIB=$L/libpqgpu_d7.so $B"
