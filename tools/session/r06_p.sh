#!/bin/bash
# round 6 session P: k_ba_emit look-back (window 16/64 predecessors, help after 24/4 polls, or the pre-pass
# bases) on cfg3 / cfg4; cfg1 kernel trace with the runtime's own kernels
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/parquet-go-1_amd/lib
V3='[{}, {"PQ_BA_PRESUM": "1"}, {"PQ_BA_PRESUM": "2"}, {}]'
tools/gpu_steps.sh \
  "200 c3 python tools/variant_probe.py --config cfg3 --variants '$V3'" \
  "200 c3lb64 env PQGPU_LIB=$L/libpqgpu_lb64.so python tools/variant_probe.py --config cfg3 --variants '[{}, {}]'" \
  "200 c3help4 env PQGPU_LIB=$L/libpqgpu_help4.so python tools/variant_probe.py --config cfg3 --variants '[{}, {}]'" \
  "200 c3lb64h4 env PQGPU_LIB=$L/libpqgpu_lb64h4.so python tools/variant_probe.py --config cfg3 --variants '[{}, {}]'" \
  "300 c4 python tools/variant_probe.py --config cfg4 --variants '[{}, {\"PQ_BA_PRESUM\": \"1\"}]'" \
  "300 c4lb64 env PQGPU_LIB=$L/libpqgpu_lb64.so python tools/variant_probe.py --config cfg4 --variants '[{}]'" \
  "200 tl1 timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl1 -o run -- python3 bench.py --config cfg1 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e"
