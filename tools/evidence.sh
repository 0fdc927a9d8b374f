#!/bin/bash
# Round evidence for the given workloads: tools/prof.sh (kernel trace + stats, FETCH_SIZE,
# WRITE_SIZE and SQ passes, each its own rocprofv3 run under its own time limit), with a
# heartbeat line every 30 s so a long workload generation is not taken for a hang.
#   tools/evidence.sh cfg1 cfg2 ...   -> gpurun_out/prof_<cfg>/ (then tools/prof_summary.py <cfg> <round>)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
( while true; do sleep 30; echo "[evidence] alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB' EXIT
for CFG in "$@"; do
  echo "[evidence] $CFG"
  tools/prof.sh $CFG || exit 1
done
