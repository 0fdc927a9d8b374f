#!/bin/bash
# round 6 session B: k_levels_seg rewrite (v2 = the default build) — GPU suite and smoke, then cfg2 per
# library (r5: round-5 kernels / v1: lean walk + LDS image / v2: table walk with lane buffers), kernels
# alone (PQ_ONE_STREAM=1) and in the default schedule; the copy-shape ubench
cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/parquet-go-1_amd/lib
B="python bench.py --no-cpu-baseline --no-e2e --steps 20 --warmup 3"
tools/gpu_steps.sh \
  "600 tests python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "120 smoke python -c 'import __graft_entry__ as g; g.smoke()'" \
  "200 b_r5_one env PQ_ONE_STREAM=1 PQGPU_LIB=$L/libpqgpu_r5.so $B" \
  "200 b_v1_one env PQ_ONE_STREAM=1 PQGPU_LIB=$L/libpqgpu_v1.so $B" \
  "200 b_v2_one env PQ_ONE_STREAM=1 $B" \
  "200 b_r5 env PQGPU_LIB=$L/libpqgpu_r5.so $B" \
  "200 b_v1 env PQGPU_LIB=$L/libpqgpu_v1.so $B" \
  "200 b_v2 $B" \
  "120 copy_shapes tools/ubench/copy_shapes"
