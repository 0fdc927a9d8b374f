#!/bin/bash
# Round-4 evidence: per workload the bench line (20 timed steps after 3 warm-ups, with the streamed
# passes and the CPU baselines) and tools/prof.sh (rocprofv3 kernel trace + stats, FETCH_SIZE,
# WRITE_SIZE, SQ passes), each under its own limit; optional extra steps appended by the caller.
# usage: tools/r04_evidence.sh <cfg>... [-- "<limit> <name> <command>"...]
cd "$(dirname "$0")/.."
steps=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do
  c=$1; shift
  steps+=("400 bench_$c python -u bench.py --config $c --steps 20 --warmup 3")
  steps+=("700 prof_$c tools/prof.sh $c")
done
[ "$1" == "--" ] && shift
exec tools/gpu_steps.sh "${steps[@]}" "$@"
