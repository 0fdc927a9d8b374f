#!/bin/bash
# Round 5 session 15: k_nest_count writes per-slot flag masks (no packed levels), k_nest_emit reads
# them (no level unpacking, no flag loop); parity, cfg4 bench, nested phase stamps, timeline.
cd "$(dirname "$0")/.."
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
T="python -u -m pytest tests/test_nested.py tests/test_struct.py tests/test_ref_goldens.py tests/test_levels_segw.py tests/test_gpu_parity.py tests/test_switches.py tests/test_ba_classes.py -m gpu -q -x --timeout 120 --timeout-method thread -rf"
tools/gpu_steps.sh \
  "400 s15_tests $T" \
  "200 s15_cfg4 $B --config cfg4" \
  "200 s15_diag_nest python -u tools/diag_nest.py" \
  "200 s15_tl_cfg4 tools/timeline.sh cfg4"
