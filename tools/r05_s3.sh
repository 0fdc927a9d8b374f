#!/bin/bash
# Round 5 session 3: byte-array ubench variants, the GPU suite with the new level defaults, cfg4
# kernel trace.
cd "$(dirname "$0")/.."
R=$(pwd)
tools/gpu_steps.sh \
  "150 s3_ba_ubench tools/ubench/ba_ubench" \
  "600 s3_gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 s3_prof_cfg4 cd /tmp && export TMPDIR=/tmp && cd $R && timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s3_prof_cfg4 -o run -- python3 bench.py --config cfg4 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
