#!/bin/bash
# round 6 session R: dictionary-only schedule (cfg1: no reset launch, no event record per decode),
# 8-group stride prelude in hyb_scan; GPU suite, cfg1/cfg3/cfg4 timelines and lines
cd "$GRAFT_REPO_ROOT"
B="python bench.py --no-cpu-baseline --no-e2e --steps 20 --warmup 3"
tools/gpu_steps.sh \
  "700 tests python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread" \
  "200 tl1 tools/timeline.sh cfg1" \
  "200 tl3 tools/timeline.sh cfg3" \
  "300 tl4 tools/timeline.sh cfg4" \
  "200 cfg1 $B --config cfg1" \
  "200 cfg3 $B --config cfg3" \
  "300 cfg4 $B --config cfg4"
