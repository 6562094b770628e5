#!/bin/bash
# Runs one gpurun call, retrying ONLY while the pool has no box / the call was
# refused for infrastructure reasons before anything ran (gpurun exit 3 or a
# "transient" verdict, nothing charged); any other result ends the loop.
#   tools/gpurun_retry.sh TIMEOUT 'command'
t=$1; shift
for k in $(seq 1 ${TRIES:-20}); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@"
  rc=$?
  st=$(python3 -c "import json; print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ $rc -ne 3 ] && [ "$st" != transient ]; then exit $rc; fi
  echo "[retry $k: rc=$rc status=$st]"; sleep ${SLEEP:-120}
done
exit 3
