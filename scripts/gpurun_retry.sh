#!/bin/bash
# Submit a gpurun call; resubmit only when the infrastructure reports a
# transient failure before anything ran (no box / box lost while preparing).
# A command that ran and failed is never resubmitted.
# usage: gpurun_retry.sh OUTFILE TIMEOUT 'command'
out=$1; lim=$2; shift 2
for attempt in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout $lim -- "$@" > $out 2>&1
  rc=$?
  if grep -q "status=transient\|no box or slot\|backing off" $out && ! grep -q "status=ok\|status=fail" $out; then
    sleep $((60 * attempt)); continue
  fi
  exit $rc
done
exit $rc
