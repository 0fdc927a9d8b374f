#!/bin/bash
# Round 5 session 5: GPU suite on the new defaults, benches, cfg2 copy NT variants, DELTA phase stamps,
# cfg2 one-stream kernel times, cfg4 trace.
cd "$(dirname "$0")/.."
R=$(pwd)
L=parquet-go-1_amd/lib
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
tools/gpu_steps.sh \
  "600 s5_gpu_tests python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -rf" \
  "200 s5_cfg2 $B --config cfg2" \
  "200 s5_cfg2_copynt1 env PQGPU_LIB=$L/libpqgpu_copynt1.so $B --config cfg2" \
  "200 s5_cfg2_copynt2 env PQGPU_LIB=$L/libpqgpu_copynt2.so $B --config cfg2" \
  "200 s5_cfg2_one env PQ_ONE_STREAM=1 $B --config cfg2" \
  "200 s5_cfg3 $B --config cfg3" \
  "200 s5_cfg4 $B --config cfg4" \
  "200 s5_cfg4_one env PQ_ONE_STREAM=1 $B --config cfg4" \
  "200 s5_diag_cfg2 python -u tools/diag.py cfg2" \
  "200 s5_prof_cfg4 cd /tmp && export TMPDIR=/tmp && cd $R && timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s5_prof_cfg4 -o run -- python3 bench.py --config cfg4 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
