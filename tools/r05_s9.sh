#!/bin/bash
# Round 5 session 9: suite (try_stride fix, DELTA-major cfg2 schedule), cfg2 bench + trace, cfg4 diag.
cd "$(dirname "$0")/.."
R=$(pwd)
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
tools/gpu_steps.sh \
  "300 s9_level_tests python -u -m pytest tests/test_levels_segw.py tests/test_switches.py tests/test_gpu_parity.py -m gpu -q -x --timeout 60 --timeout-method thread -rf" \
  "600 s9_gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 60 --timeout-method thread -rf" \
  "200 s9_cfg2 $B --config cfg2" \
  "200 s9_prof_cfg2 cd /tmp && export TMPDIR=/tmp && cd $R && timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s9_prof_cfg2 -o run -- python3 bench.py --config cfg2 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e" \
  "200 s9_diag_cfg4 python -u tools/diag.py cfg4"
