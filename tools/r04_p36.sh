#!/bin/bash
# Probe: SNAPPY long-literal bodies with one load per 16-B piece (lib oneload; lib u8: 8 pieces per
# lane in flight) against two loads per piece (the default build); parity of the one-load build first.
cd "$(dirname "$0")/.."
L=$PWD/parquet-go-1_amd/lib
exec tools/gpu_steps.sh \
 "300 snappy_tests env PQGPU_LIB=$L/libpqgpu_oneload.so python -u -m pytest tests/test_snappy.py tests/test_pipeline.py -m gpu -x -q --timeout 120 --timeout-method thread" \
 "300 snappy_tests_u8 env PQGPU_LIB=$L/libpqgpu_u8.so python -u -m pytest tests/test_snappy.py -m gpu -x -q --timeout 120 --timeout-method thread" \
 "300 p_cfg5 python -u tools/variant_probe.py --config cfg5 --variants '[{}, {}]'" \
 "300 p_cfg5_one env PQGPU_LIB=$L/libpqgpu_oneload.so python -u tools/variant_probe.py --config cfg5 --variants '[{}, {}]'" \
 "300 p_cfg5_u8 env PQGPU_LIB=$L/libpqgpu_u8.so python -u tools/variant_probe.py --config cfg5 --variants '[{}, {}]'" \
 "300 p_cfg5b python -u tools/variant_probe.py --config cfg5 --variants '[{}]'"
