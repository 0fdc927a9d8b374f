#!/bin/bash
# HBM traffic of the decode kernels from PMC counters (MI355X_MICROARCH.md §HBM):
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes (they do not fit one TCC pass),
# each pass its own run under its own time limit; then a kernel-trace --stats run of the
# same command. Results: gpurun_out/pmc_traffic/{fetch,write,stats}/...; summarised into
# profiles/ by tools/pmc_summary.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_traffic
mkdir -p $OUT
CMD="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_values|k_levels" --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $CMD > $OUT/fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_values|k_levels" --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $CMD > $OUT/write.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- $CMD > $OUT/stats.log 2>&1
