#!/bin/bash
# round 6 session Q (re-entry): GPU suite + smoke on HEAD (k_levels_seg changes after the J evidence),
# default bench line, kernel timelines of cfg3 and cfg4 for the next cuts
cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "700 tests python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread" \
  "120 smoke python -c 'import __graft_entry__ as g; g.smoke()'" \
  "300 default python bench.py --gpus 1 --steps 20 --warmup 5" \
  "200 tl3 tools/timeline.sh cfg3" \
  "300 tl4 tools/timeline.sh cfg4" \
  "200 tl1 tools/timeline.sh cfg1"
