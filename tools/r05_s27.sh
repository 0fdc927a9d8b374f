#!/bin/bash
# Round 5 session 27: timelines of cfg4 / cfg3 / cfg2 (critical paths); k_ba_emit with the first slot
# pieces loaded in pass A (P0) at 5 and 4 waves per SIMD against the default, cfg3; byte-array parity; plain-store assembly (PQ_BA_PLAIN).
cd "$(dirname "$0")/.."
L=parquet-go-1_amd/lib
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --config cfg3"
T="python -u -m pytest tests/test_ba_classes.py tests/test_dict_groups.py tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -rf"
tools/gpu_steps.sh \
  "200 s27_tl4 tools/timeline.sh cfg4" \
  "200 s27_tl3 tools/timeline.sh cfg3" \
  "200 s27_tl2 tools/timeline.sh cfg2" \
  "300 s27_tests_p0w5 env PQGPU_LIB=$L/libpqgpu_p0w5.so $T" \
  "200 s27_cfg3_base env PQGPU_LIB=$L/libpqgpu_base.so $B" \
  "200 s27_cfg3_p0w5 env PQGPU_LIB=$L/libpqgpu_p0w5.so $B" \
  "200 s27_cfg3_p0w4 env PQGPU_LIB=$L/libpqgpu_p0w4.so $B" \
  "200 s27_cfg3_base_b env PQGPU_LIB=$L/libpqgpu_base.so $B" \
  "200 s27_cfg3_p0w5_b env PQGPU_LIB=$L/libpqgpu_p0w5.so $B" \
  "300 s27_tests_plain env PQGPU_LIB=$L/libpqgpu_plain.so $T" \
  "200 s27_cfg3_plain env PQGPU_LIB=$L/libpqgpu_plain.so $B" \
  "200 s27_cfg3_plainp0w5 env PQGPU_LIB=$L/libpqgpu_plainp0w5.so $B" \
  "200 s27_cfg3_plain_b env PQGPU_LIB=$L/libpqgpu_plain.so $B"
