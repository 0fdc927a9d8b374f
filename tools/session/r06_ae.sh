#!/bin/bash
# round 6 session AE: cfg4's level walkers at wave priority 3 beside the early copies (libpqgpu_prio3.so)
cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/parquet-go-1_amd/lib
tools/gpu_steps.sh \
  "300 c4 python tools/variant_probe.py --config cfg4 --variants '[{}, {}]'" \
  "300 c4p env PQGPU_LIB=$L/libpqgpu_prio3.so python tools/variant_probe.py --config cfg4 --variants '[{}, {}]'"
