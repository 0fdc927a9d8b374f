#!/bin/bash
# rocprofv3 evidence for one bench workload (MI355X_MICROARCH.md rocprofv3 / HBM sections):
#   stats  : --kernel-trace --stats (per-kernel durations)
#   fetch  : --pmc FETCH_SIZE           (own pass: FETCH_SIZE takes 3 TCC slots)
#   write  : --pmc WRITE_SIZE           (own pass)
#   sq     : --pmc 8 SQ counters (waves, wave/busy cycles, stall buckets, LDS bank conflicts)
# Every pass is its own run under its own hard time limit; a failing pass stops the script.
# The stats pass runs the bench's own timed steps (20 after 3 warm-ups, no streamed passes): its JSON
# line (in stats.log) carries the live HIP-event kernel means that the trace averages must match.
# usage: tools/prof.sh <config> [extra bench args]   -> gpurun_out/prof_<config>/...
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
CFG=${1:-cfg2}; shift
OUT=gpurun_out/prof_$CFG
mkdir -p $OUT
CMD="python3 bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-e2e $*"
SQ="SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE"
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- $CMD > $OUT/stats.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $CMD > $OUT/fetch.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $CMD > $OUT/write.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc $SQ --output-format csv -d $OUT/sq -o run -- $CMD > $OUT/sq.log 2>&1
rc=$?
tail -n 3 $OUT/*.log
exit $rc
