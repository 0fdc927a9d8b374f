#!/bin/bash
# Round 5 session 22: k_dict_slots on the copy stream from the start; k_ba_sums with the 16 rounds'
# length gathers in flight together; parity, cfg3 / cfg4, cfg4 timeline.
cd "$(dirname "$0")/.."
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
T="python -u -m pytest tests/test_ba_classes.py tests/test_gpu_parity.py tests/test_delta_bytearray.py tests/test_plain_bytearray.py tests/test_switches.py tests/test_nested.py tests/test_struct.py tests/test_dict_groups.py tests/test_page_index.py tests/test_pipeline.py -m gpu -q -x --timeout 120 --timeout-method thread -rf"
tools/gpu_steps.sh \
  "400 s22_tests $T" \
  "200 s22_cfg3 $B --config cfg3" \
  "200 s22_cfg4 $B --config cfg4" \
  "200 s22_tl_cfg4 tools/timeline.sh cfg4"
