#!/bin/bash
# k_snappy HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) and a kernel-trace --stats run
# of the SNAPPY bench workload; summaries copied to profiles/ by hand.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_snappy
mkdir -p $OUT
CMD="python3 bench.py --codec SNAPPY --steps 3 --warmup 1 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_snappy" --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $CMD > $OUT/fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_snappy" --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $CMD > $OUT/write.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 bench.py --codec SNAPPY --steps 20 --no-cpu-baseline > $OUT/stats.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cfg2 -o run -- python3 bench.py --steps 20 --no-cpu-baseline > gpurun_out/prof_cfg2.log 2>&1
