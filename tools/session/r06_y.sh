#!/bin/bash
# round 6 session Y: serial batches' PLAIN copies beside the level kernels on counts speculated from
# the pages' value bytes (copies_early; PQ_COPY_EARLY=0: after k_bases); parity, cfg4 A/B and timeline
cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "500 tests python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread" \
  "300 c4 python tools/variant_probe.py --config cfg4 --variants '[{}, {\"PQ_COPY_EARLY\": \"0\"}, {}, {\"PQ_COPY_EARLY\": \"0\"}]'" \
  "300 tl4 tools/timeline.sh cfg4"
