#!/bin/bash
# Round 5 session 2: the byte-array gather micro-benchmark, the switch-parity suite, cfg4 with the
# definition streams on k_levels_segw.
cd "$(dirname "$0")/.."
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
tools/gpu_steps.sh \
  "120 s2_ba_ubench tools/ubench/ba_ubench" \
  "600 s2_switches python -u -m pytest tests/test_switches.py tests/test_dict_groups.py tests/test_struct.py tests/test_page_index.py -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 s2_cfg4 $B --config cfg4" \
  "200 s2_cfg4_segw2 env PQ_LV_SEGW=2 $B --config cfg4" \
  "200 s2_cfg4_segw1 env PQ_LV_SEGW=1 $B --config cfg4"
