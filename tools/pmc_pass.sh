#!/bin/bash
# One rocprofv3 PMC pass (its own run, hard time limit) over a bench workload:
#   tools/pmc_pass.sh <config> <name> <comma-separated counters>  -> gpurun_out/pmc_<config>_<name>/
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
CFG=$1; NAME=$2; CTRS=$3
OUT=gpurun_out/pmc_${CFG}_${NAME}
mkdir -p $OUT
timeout -s KILL 150 rocprofv3 --pmc $CTRS --output-format csv -d $OUT -o run -- python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/log 2>&1
rc=$?
tail -2 $OUT/log
exit $rc
