#!/bin/bash
# CPU container: one gpurun call, waiting (up to ~40 min) while the pool has no free box (a
# "transient" verdict: nothing ran, nothing charged).  Any other outcome -- success or a failure
# of the command itself -- is final.  usage: tools/gpurun_wait.sh <timeout> '<cmd>'
to=$1; cmd=$2
for i in $(seq 1 16); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd"
  rc=$?
  python3 -c "import json,sys; sys.exit(0 if json.load(open('gpurun_out/.last_call.json'))['status'] == 'transient' else 1)" || exit $rc
  sleep 150
done
exit 3
