#!/bin/bash
# round 6 session M: k_ba_emit pass-B load groups (G rounds of second slot pieces in flight) x waves per
# SIMD, on cfg3 and cfg4
cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/parquet-go-1_amd/lib
tools/gpu_steps.sh \
  "200 c3 python tools/variant_probe.py --config cfg3 --variants '[{}, {}]'" \
  "200 c3g4w4 env PQGPU_LIB=$L/libpqgpu_ba_g4w4.so python tools/variant_probe.py --config cfg3 --variants '[{}, {}]'" \
  "200 c3g8w4 env PQGPU_LIB=$L/libpqgpu_ba_g8w4.so python tools/variant_probe.py --config cfg3 --variants '[{}, {}]'" \
  "200 c3g8w5 env PQGPU_LIB=$L/libpqgpu_ba_g8w5.so python tools/variant_probe.py --config cfg3 --variants '[{}, {}]'" \
  "300 c4 python tools/variant_probe.py --config cfg4 --variants '[{}]'" \
  "300 c4g8w4 env PQGPU_LIB=$L/libpqgpu_ba_g8w4.so python tools/variant_probe.py --config cfg4 --variants '[{}]'"
