#!/bin/bash
# round 6 session X: k_ba_emit look-back window (16 / 32 / 64 predecessors per round trip), help
# after 24 / 4 polls, or the pre-pass bases (PQ_BA_PRESUM=1), on cfg3 and cfg4
cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/parquet-go-1_amd/lib
V3='[{}, {"PQ_BA_PRESUM": "1"}, {}]'
tools/gpu_steps.sh \
  "200 c3 python tools/variant_probe.py --config cfg3 --variants '$V3'" \
  "200 c3lb64 env PQGPU_LIB=$L/libpqgpu_lb64.so python tools/variant_probe.py --config cfg3 --variants '[{}, {}]'" \
  "200 c3lb32 env PQGPU_LIB=$L/libpqgpu_lb32.so python tools/variant_probe.py --config cfg3 --variants '[{}, {}]'" \
  "200 c3help4 env PQGPU_LIB=$L/libpqgpu_help4.so python tools/variant_probe.py --config cfg3 --variants '[{}, {}]'" \
  "200 c3lb64h4 env PQGPU_LIB=$L/libpqgpu_lb64h4.so python tools/variant_probe.py --config cfg3 --variants '[{}, {}]'" \
  "300 c4 python tools/variant_probe.py --config cfg4 --variants '[{}, {\"PQ_BA_PRESUM\": \"1\"}]'" \
  "300 c4lb64 env PQGPU_LIB=$L/libpqgpu_lb64.so python tools/variant_probe.py --config cfg4 --variants '[{}]'"
