#!/bin/bash
# round 6 session V: cfg4 schedules -- k_nest_pcount first, then the PLAIN copies beside k_nest_tile and
# the byte-array path after it (PQ_NEST_PCOUNT=2)
cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "300 tests python -u -m pytest tests/test_switches.py tests/test_nested.py -m gpu -q -x --timeout 120 --timeout-method thread" \
  "300 c4 python tools/variant_probe.py --config cfg4 --variants '[{}, {\"PQ_NEST_PCOUNT\": \"2\"}, {\"PQ_NEST_PCOUNT\": \"1\"}, {}, {\"PQ_NEST_PCOUNT\": \"2\"}]'" \
  "300 tl4 env PQ_NEST_PCOUNT=2 tools/timeline.sh cfg4"
