#!/bin/bash
# round 6 session K: DELTA window size (8 / 16 / 24 KB: fewer per-window drains of the output stores),
# on cfg2 and cfg5; k_levels_seg phase stamps
cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/parquet-go-1_amd/lib
V='[{}, {"PQ_ONE_STREAM": 1}]'
tools/gpu_steps.sh \
  "200 w8 python tools/variant_probe.py --config cfg2 --variants '$V'" \
  "200 w16 env PQGPU_LIB=$L/libpqgpu_win16.so python tools/variant_probe.py --config cfg2 --variants '$V'" \
  "200 w24 env PQGPU_LIB=$L/libpqgpu_win24.so python tools/variant_probe.py --config cfg2 --variants '$V'" \
  "200 w8a env PQ_ONE_STREAM=1 python tools/variant_probe.py --config cfg2 --shape a,req --variants '[{}]'" \
  "200 w16a env PQ_ONE_STREAM=1 PQGPU_LIB=$L/libpqgpu_win16.so python tools/variant_probe.py --config cfg2 --shape a,req --variants '[{}]'" \
  "300 c5w8 python tools/variant_probe.py --config cfg5 --variants '[{}]'" \
  "300 c5w16 env PQGPU_LIB=$L/libpqgpu_win16.so python tools/variant_probe.py --config cfg5 --variants '[{}]'" \
  "200 diag python tools/diag.py cfg2"
