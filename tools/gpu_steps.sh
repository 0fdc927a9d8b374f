#!/bin/bash
# Run GPU steps in order, each under its own time limit. A step that fails
# normally (exit 1, e.g. a test failure) lets the next one run; a fault,
# abort, segfault or time limit (any other non-zero status) stops the script.
# usage: tools/gpu_steps.sh "<limit_s> <name> <command>" ...
mkdir -p gpurun_out
for step in "$@"; do
  limit=${step%% *}; rest=${step#* }; name=${rest%% *}; cmd=${rest#* }
  echo "=== $name (limit ${limit}s): $cmd"
  timeout -k 10 "$limit" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  if grep -qiE "illegal memory access|memory access fault|hipErrorLaunchFailure|HSA_STATUS_ERROR|core dumped" "gpurun_out/$name.log"; then
    echo "stopping after $name: GPU fault reported"; exit 3
  fi
done
