#!/bin/bash
# round 6 session U: k_levels_hyb with the 8-group stride prelude (PQ_HYB_PRE=1) against the windowed
# walk alone (libpqgpu_nopre.so); nested parity
cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/parquet-go-1_amd/lib
tools/gpu_steps.sh \
  "300 tests python -u -m pytest tests/test_nested.py tests/test_struct.py tests/test_levels_segw.py tests/test_gpu_parity.py tests/test_switches.py -m gpu -q -x --timeout 120 --timeout-method thread" \
  "300 c4 python tools/variant_probe.py --config cfg4 --variants '[{}, {}, {\"PQ_ONE_STREAM\": \"1\"}]'" \
  "300 c4nopre env PQGPU_LIB=$L/libpqgpu_nopre.so python tools/variant_probe.py --config cfg4 --variants '[{}, {}, {\"PQ_ONE_STREAM\": \"1\"}]'"
