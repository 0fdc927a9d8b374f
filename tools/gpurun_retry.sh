#!/bin/bash
# Call gpurun; if the box could not be prepared (status=transient, nothing ran,
# nothing charged) or no box was free (exit 3), wait (the backoff gpurun names, else 60 s) and
# call again (TRIES, default 4). A command that actually ran is never repeated.
for i in $(seq 1 ${TRIES:-4}); do
  out=$(/usr/local/graft/bin/gpurun "$@" 2>&1); rc=$?
  echo "$out" | grep -v "^W2026\|^E2026\|every call sends"
  if echo "$out" | grep -q "status=transient" || [ $rc -eq 3 ]; then
    w=$(echo "$out" | grep -o "retry in [0-9]*s" | grep -o "[0-9]*" | head -1)
    sleep $(( ${w:-60} + 5 ))
    continue
  fi
  exit $rc
done
exit 3
