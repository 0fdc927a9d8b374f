#!/bin/bash
# Round 5 session 14: the nested chunk scan by k_nest_count's last tile per chunk (no k_nest_scan
# launch), the byte-array path ahead of the copy join; parity, cfg4 bench and kernel timeline.
cd "$(dirname "$0")/.."
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
T="python -u -m pytest tests/test_nested.py tests/test_struct.py tests/test_ref_goldens.py tests/test_levels_segw.py tests/test_gpu_parity.py tests/test_switches.py tests/test_ba_classes.py -m gpu -q -x --timeout 120 --timeout-method thread -rf"
tools/gpu_steps.sh \
  "400 s14_tests $T" \
  "200 s14_cfg4 $B --config cfg4" \
  "200 s14_tl_cfg4 tools/timeline.sh cfg4"
