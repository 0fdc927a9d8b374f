#!/bin/bash
# Probe: dictionary run cursor in registers (default) vs a run-table read per value (lib nocur).
cd "$(dirname "$0")/.."
L=$PWD/parquet-go-1_amd/lib
exec tools/gpu_steps.sh \
 "300 dict_tests python -u -m pytest tests/test_gpu_parity.py tests/test_snappy.py tests/test_stride.py tests/test_ba_classes.py -m gpu -x -q --timeout 120 --timeout-method thread" \
 "300 p_cfg5 python -u tools/variant_probe.py --config cfg5 --variants '[{}, {}]'" \
 "300 p_cfg5_nocur env PQGPU_LIB=$L/libpqgpu_nocur.so python -u tools/variant_probe.py --config cfg5 --variants '[{}, {}]'" \
 "200 p_cfg1 python -u tools/variant_probe.py --config cfg1 --variants '[{}, {}]'" \
 "200 p_cfg1_nocur env PQGPU_LIB=$L/libpqgpu_nocur.so python -u tools/variant_probe.py --config cfg1 --variants '[{}, {}]'"
