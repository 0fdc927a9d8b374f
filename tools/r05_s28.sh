#!/bin/bash
# Round 5 session 28: the fused nested pass (k_nest_tile) -- full GPU suite with it, cfg4 A/B against
# the two passes (PQ_NEST_FUSED=0); kernel timelines of cfg4 / cfg3 / cfg2; k_ba_emit variants on cfg3:
# first slot pieces in pass A (P0) at 5 / 4 waves per SIMD, plain-store assembly (PLAIN).
cd "$(dirname "$0")/.."
L=parquet-go-1_amd/lib
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
T="python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf"
TB="python -u -m pytest tests/test_ba_classes.py tests/test_dict_groups.py tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -rf"
tools/gpu_steps.sh \
  "400 s28_tests $T" \
  "200 s28_cfg4_fused $B --config cfg4" \
  "200 s28_cfg4_twopass env PQ_NEST_FUSED=0 $B --config cfg4" \
  "200 s28_cfg4_fused_b $B --config cfg4" \
  "200 s28_tl4 tools/timeline.sh cfg4" \
  "200 s28_tl3 tools/timeline.sh cfg3" \
  "200 s28_tl2 tools/timeline.sh cfg2" \
  "300 s28_tests_p0w5 env PQGPU_LIB=$L/libpqgpu_p0w5.so $TB" \
  "300 s28_tests_plain env PQGPU_LIB=$L/libpqgpu_plain.so $TB" \
  "200 s28_cfg3_base env PQGPU_LIB=$L/libpqgpu_base.so $B --config cfg3" \
  "200 s28_cfg3_p0w5 env PQGPU_LIB=$L/libpqgpu_p0w5.so $B --config cfg3" \
  "200 s28_cfg3_p0w4 env PQGPU_LIB=$L/libpqgpu_p0w4.so $B --config cfg3" \
  "200 s28_cfg3_plain env PQGPU_LIB=$L/libpqgpu_plain.so $B --config cfg3" \
  "200 s28_cfg3_plainp0w5 env PQGPU_LIB=$L/libpqgpu_plainp0w5.so $B --config cfg3" \
  "200 s28_cfg3_base_b env PQGPU_LIB=$L/libpqgpu_base.so $B --config cfg3" \
  "200 s28_cfg3_plain_b env PQGPU_LIB=$L/libpqgpu_plain.so $B --config cfg3"
