#!/bin/bash
# Round-4 session: fused nested pipeline (k_nest_count / k_nest_emit over fill tiles) parity,
# then the cfg4 probe.
cd "$(dirname "$0")/.."
exec tools/gpu_steps.sh \
  "300 t_nest python -u -m pytest tests/test_nested.py tests/test_struct.py tests/test_levels_segw.py tests/test_gpu_parity.py tests/test_refwriter.py tests/test_ref_goldens.py tests/test_pipeline.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "200 probe_cfg4 python -u tools/variant_probe.py --config cfg4 --variants '[{}, {\"PQ_BA_PRESUM\": \"1\"}]'" \
  "120 probe_cfg2 python -u tools/variant_probe.py --config cfg2 --variants '[{}]'" \
  "$@"
