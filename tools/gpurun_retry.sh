#!/bin/bash
# Host-side helper: submit one gpurun call and resubmit it only when the pool
# reports a transient (no box / box lost while being prepared: nothing of the
# command ran).  Any status other than "transient" -- including a failure of
# the command itself -- ends the loop.  At most 8 submissions, 150 s apart.
#   tools/gpurun_retry.sh <timeout> '<command>'
to=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  [ "$st" = "transient" ] || [ $rc -eq 3 ] || exit $rc
  echo "[retry] transient ($i), waiting"
  sleep 150
done
exit 3
