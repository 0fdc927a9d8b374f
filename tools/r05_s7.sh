#!/bin/bash
# Round 5 session 7: suite on the new defaults (stride walker takes isolated short runs, NT copies),
# benches, cfg4 trace, k_levels_seg ablations on cfg2 (one stream).
cd "$(dirname "$0")/.."
R=$(pwd)
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
tools/gpu_steps.sh \
  "600 s7_gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 s7_cfg2 $B --config cfg2" \
  "200 s7_cfg4 $B --config cfg4" \
  "300 s7_cfg5 $B --config cfg5" \
  "200 s7_prof_cfg4 cd /tmp && export TMPDIR=/tmp && cd $R && timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s7_prof_cfg4 -o run -- python3 bench.py --config cfg4 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e" \
  "200 s7_ablate_cfg2 env PQ_ONE_STREAM=1 python -u tools/diag_ablate.py cfg2 0,1048576,2097152,4194304"
