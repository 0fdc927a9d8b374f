#!/bin/bash
# round 6 session Z: where cfg4's early copies go -- at the start (1), enqueued after the level kernels (2),
# beside k_nest_tile (3), after k_bases (0)
cd "$GRAFT_REPO_ROOT"
V='[{}, {"PQ_COPY_EARLY": "2"}, {"PQ_COPY_EARLY": "3"}, {"PQ_COPY_EARLY": "0"}, {}, {"PQ_COPY_EARLY": "2"}, {"PQ_COPY_EARLY": "3"}]'
tools/gpu_steps.sh \
  "300 tests python -u -m pytest tests/test_nested.py tests/test_struct.py -m gpu -q -x --timeout 120 --timeout-method thread" \
  "300 c4 python tools/variant_probe.py --config cfg4 --variants '$V'"
