#!/bin/bash
# round 6 session S: bench timed region ends at pqgpu_batch_wait; cfg1 (dictionary-only schedule)
# and cfg2 lines, ba/dict GPU tests
cd "$GRAFT_REPO_ROOT"
B="python bench.py --no-cpu-baseline --no-e2e --steps 20 --warmup 3"
tools/gpu_steps.sh \
  "300 tests python -u -m pytest tests/test_gpu_parity.py tests/test_capi.py tests/test_switches.py -m gpu -q -x --timeout 120 --timeout-method thread" \
  "200 cfg1 $B --config cfg1" \
  "200 cfg1b $B --config cfg1 --steps 200" \
  "200 cfg1off env PQ_DICT_ONLY=0 $B --config cfg1" \
  "300 cfg2 $B --config cfg2"
