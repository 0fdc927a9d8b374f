#!/bin/bash
# round 6 session AB: DELTA pages wait for the prefetched window before issuing the window's output
# stores (PQ_DELTA_EARLYWAIT=1, libpqgpu_ew.so) against the wait at the window switch
cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/parquet-go-1_amd/lib
V='[{}, {}, {"PQ_ONE_STREAM": "1"}]'
tools/gpu_steps.sh \
  "200 c2 python tools/variant_probe.py --config cfg2 --variants '$V'" \
  "200 c2ew env PQGPU_LIB=$L/libpqgpu_ew.so python tools/variant_probe.py --config cfg2 --variants '$V'" \
  "200 c2b python tools/variant_probe.py --config cfg2 --variants '[{}]'" \
  "200 c2ewb env PQGPU_LIB=$L/libpqgpu_ew.so python tools/variant_probe.py --config cfg2 --variants '[{}]'" \
  "300 tew env PQGPU_LIB=$L/libpqgpu_ew.so python -u -m pytest tests/test_delta_shapes.py tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread"
