#!/bin/bash
# Round 5 session 6: is the stride prelude effective on cfg4's repetition streams (k_levels)?
cd "$(dirname "$0")/.."
R=$(pwd)
L=parquet-go-1_amd/lib
P="cd /tmp && export TMPDIR=/tmp && cd $R && timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv"
C="python3 bench.py --config cfg4 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
tools/gpu_steps.sh \
  "200 s6_prof_stride $P -d gpurun_out/s6_prof_stride -o run -- $C" \
  "200 s6_prof_nostride export PQGPU_LIB=$R/$L/libpqgpu_nostride.so && $P -d gpurun_out/s6_prof_nostride -o run -- $C" \
  "200 s6_diag_cfg4 python -u tools/diag.py cfg4"
