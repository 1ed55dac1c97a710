#!/bin/bash
# Retry gpurun only when the pool reports a transient box-preparation failure (nothing ran,
# nothing charged); never retries a command that actually ran.
# usage: tools/gpurun_retry.sh TIMEOUT 'command'
T=$1; shift
for attempt in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  st=$(python3 -c "import json; print(json.load(open('gpurun_out/.last_call.json'))['status'])" 2>/dev/null)
  if [ "$st" != "transient" ] && [ $rc -ne 3 ]; then exit $rc; fi
  echo "[retry] transient/no box (attempt $attempt), sleeping"; sleep $((60 * attempt))
done
exit 3
