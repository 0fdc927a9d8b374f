#!/bin/bash
# Probe: byte-wide dictionary indices read as LDS bytes (default) vs the generic bit funnel (lib
# nobyte); phase stamps of k_values_dict2 on cfg5 (diagnostic library).
cd "$(dirname "$0")/.."
L=$PWD/parquet-go-1_amd/lib
exec tools/gpu_steps.sh \
 "300 dict_tests python -u -m pytest tests/test_gpu_parity.py tests/test_snappy.py -m gpu -x -q --timeout 120 --timeout-method thread" \
 "300 p_cfg5 python -u tools/variant_probe.py --config cfg5 --variants '[{}, {}]'" \
 "300 p_cfg5_nobyte env PQGPU_LIB=$L/libpqgpu_nobyte.so python -u tools/variant_probe.py --config cfg5 --variants '[{}, {}]'" \
 "200 diag_cfg5 python -u tools/diag.py cfg5"
