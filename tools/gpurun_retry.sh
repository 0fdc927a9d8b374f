#!/bin/bash
# Call gpurun; if the box could not be prepared (status=transient, nothing ran,
# nothing charged) or no box was free (exit 3), wait and call again (max 4 tries).
# A command that actually ran is never repeated.
for i in $(seq 1 ${TRIES:-4}); do
  out=$(/usr/local/graft/bin/gpurun "$@" 2>&1); rc=$?
  echo "$out" | grep -v "^W2026\|^E2026"
  if echo "$out" | grep -q "status=transient" || [ $rc -eq 3 ]; then sleep 40; continue; fi
  exit $rc
done
exit 3
