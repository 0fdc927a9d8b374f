#!/bin/bash
# round 6 session E: why k_levels_seg v2 is slow in the production build (kernel trace; the diag build
# without stamps), then the cfg2 schedule probes (session D) on the v1 level kernel
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/parquet-go-1_amd/lib
B="python bench.py --no-cpu-baseline --no-e2e --steps 5 --warmup 2"
V='[{}, {"PQ_PLAIN_TILE_B": 8192}, {"PQ_PLAIN_TILE_B": 16384}, {"PQ_PLAIN_TILE_B": 32768}, {"PQ_SEG_GRID": 512}, {"PQ_SEG_GRID": 1024}, {"PQ_ONE_STREAM": 1}, {"PQ_ONE_STREAM": 1, "PQ_PLAIN_TILE_B": 16384}]'
VS='[{}, {"PQ_PLAIN_TILE_B": 16384}]'
tools/gpu_steps.sh \
  "200 trace_v2 env PQ_ONE_STREAM=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_v2 -o run -- $B" \
  "200 diaglib_one env PQ_ONE_STREAM=1 PQGPU_LIB=$L/libpqgpu_diag.so $B" \
  "300 probe env PQGPU_LIB=$L/libpqgpu_v1.so python tools/variant_probe.py --config cfg2 --variants '$V'" \
  "200 shape_a env PQGPU_LIB=$L/libpqgpu_v1.so python tools/variant_probe.py --config cfg2 --shape a,req --variants '$VS'" \
  "200 shape_b env PQGPU_LIB=$L/libpqgpu_v1.so python tools/variant_probe.py --config cfg2 --shape b,req --variants '$VS'" \
  "200 shape_req env PQGPU_LIB=$L/libpqgpu_v1.so python tools/variant_probe.py --config cfg2 --shape req --variants '$VS'"
