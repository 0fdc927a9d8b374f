#!/bin/bash
# Probe: dictionary tiles grouped three to a workgroup (default) vs two (PQ_DICT_GROUP=2) vs one.
cd "$(dirname "$0")/.."
exec tools/gpu_steps.sh \
 "300 dict_tests python -u -m pytest tests/test_gpu_parity.py tests/test_snappy.py -m gpu -x -q --timeout 120 --timeout-method thread" \
 "300 p_cfg5 python -u tools/variant_probe.py --config cfg5 --variants '[{}, {\"PQ_DICT_GROUP\": \"2\"}, {\"PQ_DICT_PAIR\": \"0\"}, {}, {\"PQ_DICT_GROUP\": \"2\"}]'" \
 "200 diag_cfg5 python -u tools/diag.py cfg5"
