#!/bin/bash
# Probe: paired dictionary tiles (k_values_dict2) on cfg5, against PQ_DICT_PAIR=0; parity first.
cd "$(dirname "$0")/.."
exec tools/gpu_steps.sh \
 "300 dict_tests python -u -m pytest tests/test_gpu_parity.py tests/test_snappy.py tests/test_stride.py -m gpu -x -q --timeout 120 --timeout-method thread" \
 "300 p_cfg5 python -u tools/variant_probe.py --config cfg5 --variants '[{}, {\"PQ_DICT_PAIR\": \"0\"}, {}, {\"PQ_DICT_PAIR\": \"0\"}]'" \
 "200 p_cfg1 python -u tools/variant_probe.py --config cfg1 --variants '[{}, {\"PQ_DICT_PAIR\": \"1\"}]'"
