#!/bin/bash
# Round 5 session 8: k_levels_hyb for repetition streams: level tests, suite, cfg4 bench + trace.
cd "$(dirname "$0")/.."
R=$(pwd)
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
tools/gpu_steps.sh \
  "300 s8_level_tests python -u -m pytest tests/test_levels_segw.py tests/test_nested.py tests/test_struct.py tests/test_ref_goldens.py tests/test_switches.py -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "600 s8_gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 s8_cfg4 $B --config cfg4" \
  "200 s8_prof_cfg2 cd /tmp && export TMPDIR=/tmp && cd $R && timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s8_prof_cfg2 -o run -- python3 bench.py --config cfg2 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e" \
  "200 s8_prof_cfg4 cd /tmp && export TMPDIR=/tmp && cd $R && timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s8_prof_cfg4 -o run -- python3 bench.py --config cfg4 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
