#!/bin/bash
# round 6 session O: DELTA loader wave, block parse moved to waves 1-3 — parity, cfg2 vs the previous build
cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/parquet-go-1_amd/lib
tools/gpu_steps.sh \
  "400 tests python -u -m pytest tests/test_delta_shapes.py tests/test_gpu_parity.py tests/test_delta_bytearray.py -m gpu -q --timeout 120 --timeout-method thread" \
  "200 c2 python tools/variant_probe.py --config cfg2 --variants '[{}, {\"PQ_ONE_STREAM\": 1}, {}]'" \
  "200 c2prev env PQGPU_LIB=$L/libpqgpu_prev.so python tools/variant_probe.py --config cfg2 --variants '[{}, {\"PQ_ONE_STREAM\": 1}, {}]'" \
  "200 a_req env PQ_ONE_STREAM=1 python tools/variant_probe.py --config cfg2 --shape a,req --variants '[{}]'" \
  "200 diag python tools/diag.py cfg2" \
  "200 diag_ba python tools/diag_ba.py cfg3"
