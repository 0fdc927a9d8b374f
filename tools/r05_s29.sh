#!/bin/bash
# Round 5 session 29: k_nest_tile after the look-back fix (a predecessor caught between its aggregates
# and its inclusive prefixes is read again) with a bounds guard; nested / struct / switch tests, cfg4
# A/B fused vs two passes; merged scan + slot launch (k_scan_slots) on cfg3; timelines; k_ba_emit
# variants (P0, PLAIN) on cfg3.
cd "$(dirname "$0")/.."
L=parquet-go-1_amd/lib
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
TN="python -u -m pytest tests/test_nested.py tests/test_struct.py -m gpu -q -x --timeout 120 --timeout-method thread -rf"
TB="python -u -m pytest tests/test_ba_classes.py tests/test_dict_groups.py tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -rf"
tools/gpu_steps.sh \
  "300 s29_tests_nested $TN" \
  "200 s29_cfg4_fused env PQ_NEST_FUSED=1 $B --config cfg4" \
  "200 s29_cfg4_twopass env PQ_NEST_FUSED=0 $B --config cfg4" \
  "200 s29_cfg4_fused_b env PQ_NEST_FUSED=1 $B --config cfg4" \
  "300 s29_tests_all python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 s29_cfg3_scanslots $B --config cfg3" \
  "200 s29_cfg3_ownslots env PQ_SCAN_SLOTS=0 $B --config cfg3" \
  "200 s29_tl4 env PQ_NEST_FUSED=1 tools/timeline.sh cfg4" \
  "200 s29_tl3 tools/timeline.sh cfg3" \
  "200 s29_tl2 tools/timeline.sh cfg2" \
  "300 s29_tests_p0w5 env PQGPU_LIB=$L/libpqgpu_p0w5.so $TB" \
  "300 s29_tests_plain env PQGPU_LIB=$L/libpqgpu_plain.so $TB" \
  "200 s29_cfg3_base env PQGPU_LIB=$L/libpqgpu_base.so $B --config cfg3" \
  "200 s29_cfg3_p0w5 env PQGPU_LIB=$L/libpqgpu_p0w5.so $B --config cfg3" \
  "200 s29_cfg3_plain env PQGPU_LIB=$L/libpqgpu_plain.so $B --config cfg3" \
  "200 s29_cfg3_plainp0w5 env PQGPU_LIB=$L/libpqgpu_plainp0w5.so $B --config cfg3" \
  "200 s29_cfg3_p0w4 env PQGPU_LIB=$L/libpqgpu_p0w4.so $B --config cfg3" \
  "200 s29_cfg3_base_b env PQGPU_LIB=$L/libpqgpu_base.so $B --config cfg3"
