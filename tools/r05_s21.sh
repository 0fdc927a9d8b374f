#!/bin/bash
# Round 5 session 21: cfg4 byte-array tile bases by look-back (PQ_BA_PRESUM=0) or the pre-pass for the
# LDS-slot class only (2) against the default pre-pass (1 beside nested work); timelines.
cd "$(dirname "$0")/.."
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --config cfg4"
tools/gpu_steps.sh \
  "200 s21_cfg4 $B" \
  "200 s21_cfg4_p0 env PQ_BA_PRESUM=0 $B" \
  "200 s21_cfg4_p2 env PQ_BA_PRESUM=2 $B" \
  "200 s21_cfg4_b $B" \
  "200 s21_tl_p0 env PQ_BA_PRESUM=0 tools/timeline.sh cfg4"
