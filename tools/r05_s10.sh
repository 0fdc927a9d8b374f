#!/bin/bash
# Round 5 session 10: walker-counted level streams (k_bases right after the level kernels, fill and
# nested kernels beside the values path): parity suite, cfg4 bench + trace.
cd "$(dirname "$0")/.."
R=$(pwd)
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
tools/gpu_steps.sh \
  "300 s10_level_tests python -u -m pytest tests/test_levels_segw.py tests/test_nested.py tests/test_struct.py tests/test_ref_goldens.py tests/test_switches.py tests/test_gpu_parity.py -m gpu -q -x --timeout 60 --timeout-method thread -rf" \
  "600 s10_gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 60 --timeout-method thread -rf" \
  "200 s10_cfg4 $B --config cfg4" \
  "200 s10_prof_cfg4 cd /tmp && export TMPDIR=/tmp && cd $R && timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s10_prof_cfg4 -o run -- python3 bench.py --config cfg4 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
