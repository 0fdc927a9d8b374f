#!/bin/bash
# Round 5 session 24: k_nest_count per list-level group (compile-time counters: unrolled masks, 2 C wave
# sums instead of 18), k_nest_emit's group loop over the groups with a bitmap of their own; parity,
# same-box cfg4 against the previous build, stamps.
cd "$(dirname "$0")/.."
L=parquet-go-1_amd/lib
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --config cfg4"
T="python -u -m pytest tests/test_nested.py tests/test_struct.py tests/test_ref_goldens.py tests/test_levels_segw.py tests/test_gpu_parity.py tests/test_switches.py -m gpu -q -x --timeout 120 --timeout-method thread -rf"
tools/gpu_steps.sh \
  "400 s24_tests $T" \
  "200 s24_cfg4 $B" \
  "200 s24_cfg4_base env PQGPU_LIB=$L/libpqgpu_base.so $B" \
  "200 s24_cfg4_b $B" \
  "200 s24_cfg4_base_b env PQGPU_LIB=$L/libpqgpu_base.so $B" \
  "200 s24_diag_nest python -u tools/diag_nest.py"
