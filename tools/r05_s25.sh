#!/bin/bash
# Round 5 session 25: k_nest_emit loads its halves' entry bases up front; parity, cfg4 against the
# session-23 build (base).
cd "$(dirname "$0")/.."
L=parquet-go-1_amd/lib
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --config cfg4"
T="python -u -m pytest tests/test_nested.py tests/test_struct.py tests/test_ref_goldens.py tests/test_levels_segw.py -m gpu -q -x --timeout 120 --timeout-method thread -rf"
tools/gpu_steps.sh \
  "400 s25_tests $T" \
  "200 s25_cfg4 $B" \
  "200 s25_cfg4_base env PQGPU_LIB=$L/libpqgpu_base.so $B" \
  "200 s25_cfg4_b $B"
