#!/bin/bash
# Round 5 session 26: kernel timelines of cfg4 / cfg3 / cfg2 with the current build (critical paths).
cd "$(dirname "$0")/.."
tools/gpu_steps.sh \
  "200 s26_tl4 tools/timeline.sh cfg4" \
  "200 s26_tl3 tools/timeline.sh cfg3" \
  "200 s26_tl2 tools/timeline.sh cfg2"
