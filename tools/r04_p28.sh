#!/bin/bash
# Probe: k_ba_emit slot assembly without masks (default) against the masked variant (lib mask).
cd "$(dirname "$0")/.."
L=$PWD/parquet-go-1_amd/lib
exec tools/gpu_steps.sh \
 "300 ba_tests python -u -m pytest tests/test_ba_classes.py tests/test_gpu_parity.py tests/test_nested.py tests/test_struct.py -m gpu -x -q --timeout 120 --timeout-method thread" \
 "200 p_def python -u tools/variant_probe.py --config cfg3 --variants '[{}, {}]'" \
 "200 p_mask env PQGPU_LIB=$L/libpqgpu_mask.so python -u tools/variant_probe.py --config cfg3 --variants '[{}, {}]'" \
 "200 p_def4 python -u tools/variant_probe.py --config cfg4 --variants '[{}, {\"PQ_ONE_STREAM\": \"1\"}]'" \
 "200 p_mask4 env PQGPU_LIB=$L/libpqgpu_mask.so python -u tools/variant_probe.py --config cfg4 --variants '[{}, {\"PQ_ONE_STREAM\": \"1\"}]'"
