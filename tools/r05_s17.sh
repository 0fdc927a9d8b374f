#!/bin/bash
# Round 5 session 17: cfg2 A/B on one box: validity bitmaps zeroed on the level stream (split) or
# with the other resets on the batch stream (PQ_RESET_SPLIT=0), each twice, alternating.
cd "$(dirname "$0")/.."
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --config cfg2"
tools/gpu_steps.sh \
  "200 s17_split_a $B" \
  "200 s17_nosplit_a env PQ_RESET_SPLIT=0 $B" \
  "200 s17_split_b $B" \
  "200 s17_nosplit_b env PQ_RESET_SPLIT=0 $B" \
  "200 s17_tl_nosplit env PQ_RESET_SPLIT=0 tools/timeline.sh cfg2"
