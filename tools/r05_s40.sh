#!/bin/bash
# Round 5 session 40: cfg4 with the PLAIN copies after the whole byte-array path on the batch stream
# (PQ_COPY_AFTER_SCAN=2) against after the run scan (1, beside k_ba_emit) and beside the scan (0).
cd "$(dirname "$0")/.."
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
tools/gpu_steps.sh \
  "200 s40_cfg4_after_ba env PQ_COPY_AFTER_SCAN=2 $B --config cfg4" \
  "200 s40_cfg4_after_scan env PQ_COPY_AFTER_SCAN=1 $B --config cfg4" \
  "200 s40_cfg4_beside env PQ_COPY_AFTER_SCAN=0 $B --config cfg4" \
  "200 s40_cfg4_after_ba_b env PQ_COPY_AFTER_SCAN=2 $B --config cfg4" \
  "200 s40_cfg4_beside_b env PQ_COPY_AFTER_SCAN=0 $B --config cfg4" \
  "200 s40_tests env PQ_COPY_AFTER_SCAN=2 python -u -m pytest tests/test_gpu_parity.py tests/test_nested.py tests/test_struct.py tests/test_ba_classes.py -m gpu -q -x --timeout 120 --timeout-method thread -rf"
