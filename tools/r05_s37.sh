#!/bin/bash
# Round 5 session 37: cfg5 schedules -- the DELTA pages on their own stream beside the dictionary tiles
# (PQ_DELTA_SIDE=1) and the column-group pipeline (PQ_SNAPPY_GROUPS=2) against the default (every
# launch on the batch stream); cfg4 with one nested tile per workgroup again, and k_nest_tile's
# look-back polling without s_sleep (nosleep) / with a 64-tile window and no sleep (w64ns).
cd "$(dirname "$0")/.."
L=parquet-go-1_amd/lib
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
tools/gpu_steps.sh \
  "200 s37_tests python -u -m pytest tests/test_nested.py tests/test_struct.py tests/test_switches.py -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 s37_cfg4 $B --config cfg4" \
  "200 s37_cfg4_nosleep env PQGPU_LIB=$L/libpqgpu_nosleep.so $B --config cfg4" \
  "200 s37_cfg4_w64ns env PQGPU_LIB=$L/libpqgpu_w64ns.so $B --config cfg4" \
  "200 s37_cfg4_b $B --config cfg4" \
  "300 s37_cfg5 $B --config cfg5" \
  "300 s37_cfg5_side env PQ_DELTA_SIDE=1 $B --config cfg5" \
  "300 s37_cfg5_g2 env PQ_SNAPPY_GROUPS=2 $B --config cfg5"
