#!/bin/bash
# variant probes (tools/variant_probe.py) then optional rocprof evidence, each step under its own limit
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
CFG=${CFG:-cfg2}
timeout -k 10 ${PROBE_LIMIT:-400} python -u tools/variant_probe.py --config $CFG --variants "$VARIANTS" > gpurun_out/probe_$CFG.jsonl 2> gpurun_out/probe_$CFG.err
rc=$?; cat gpurun_out/probe_$CFG.jsonl; tail -5 gpurun_out/probe_$CFG.err
[ $rc -ne 0 ] && exit $rc
if [ -n "$PROF" ]; then tools/prof.sh $CFG || exit $?; fi
exit 0
