#!/bin/bash
# round 6 session AC: cfg5's run scan beside the DELTA pages (PQ_SCAN_SIDE=1), with the dictionary tiles
# too (2), or after them (0)
cd "$GRAFT_REPO_ROOT"
V='[{}, {"PQ_SCAN_SIDE": "0"}, {"PQ_SCAN_SIDE": "2"}, {}, {"PQ_SCAN_SIDE": "0"}, {"PQ_SCAN_SIDE": "2"}]'
tools/gpu_steps.sh \
  "300 tests python -u -m pytest tests/test_gpu_parity.py tests/test_snappy.py tests/test_dict_groups.py -m gpu -q -x --timeout 120 --timeout-method thread" \
  "400 c5 python tools/variant_probe.py --config cfg5 --variants '$V'"
