#!/bin/bash
# Submit one gpurun command, resubmitting it only while the pool reports that nothing ran (no free box
# or slot, or an infrastructure back-off: status "transient", nothing charged). A command that ran —
# whatever its result — is never resubmitted.  usage: tools/gpurun_wait.sh <timeout_s> <script> [tries]
t=$1; cmd=$2; tries=${3:-12}
for i in $(seq 1 "$tries"); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$cmd"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$st" != "transient" ]; then exit $rc; fi
  echo "[gpurun_wait] nothing ran (attempt $i): waiting 90 s"
  sleep 90
done
exit 3
