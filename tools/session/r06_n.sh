#!/bin/bash
# round 6 session N: DELTA pages with wave 0 as the LDS-DMA window loader (no store drains) — DELTA
# parity, then cfg2 / cfg5 against the previous build, DELTA stamps
cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/parquet-go-1_amd/lib
tools/gpu_steps.sh \
  "400 tests python -u -m pytest tests/test_delta_shapes.py tests/test_gpu_parity.py tests/test_switches.py tests/test_refwriter.py tests/test_delta_bytearray.py -m gpu -q --timeout 120 --timeout-method thread" \
  "200 c2 python tools/variant_probe.py --config cfg2 --variants '[{}, {\"PQ_ONE_STREAM\": 1}, {}]'" \
  "200 c2prev env PQGPU_LIB=$L/libpqgpu_prev.so python tools/variant_probe.py --config cfg2 --variants '[{}, {\"PQ_ONE_STREAM\": 1}, {}]'" \
  "200 a_req env PQ_ONE_STREAM=1 python tools/variant_probe.py --config cfg2 --shape a,req --variants '[{}]'" \
  "200 a_req_prev env PQ_ONE_STREAM=1 PQGPU_LIB=$L/libpqgpu_prev.so python tools/variant_probe.py --config cfg2 --shape a,req --variants '[{}]'" \
  "300 c5 python tools/variant_probe.py --config cfg5 --variants '[{}]'" \
  "300 c5prev env PQGPU_LIB=$L/libpqgpu_prev.so python tools/variant_probe.py --config cfg5 --variants '[{}]'" \
  "200 diag python tools/diag.py cfg2"
