#!/bin/bash
# Run one gpurun call; when it did not start (no free box / slot: status
# "transient", nothing ran, nothing charged) try again after a pause, at most
# $TRIES times.  A call that ran -- whatever its outcome -- is never repeated.
#   tools/gpurun_retry.sh TIMEOUT 'command'
T=$1; shift
TRIES=${TRIES:-8}
for i in $(seq 1 $TRIES); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('/root/repo/gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$st" != "transient" ]; then exit $rc; fi
  echo "[retry] no box (attempt $i), waiting"; sleep ${RETRY_SLEEP:-150}
done
exit 3
