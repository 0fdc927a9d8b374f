#!/bin/bash
# round 6 session L: k_levels_seg with the pipelined emission step and the unrolled stage load — level
# parity, cfg2 line, phase stamps
cd "$GRAFT_REPO_ROOT"
tools/gpu_steps.sh \
  "400 tests python -u -m pytest tests/test_levels_seg.py tests/test_gpu_parity.py tests/test_switches.py tests/test_refwriter.py tests/test_struct.py -m gpu -q --timeout 120 --timeout-method thread" \
  "200 probe python tools/variant_probe.py --config cfg2 --variants '[{}, {\"PQ_ONE_STREAM\": 1}, {}]'" \
  "200 diag python tools/diag.py cfg2"
