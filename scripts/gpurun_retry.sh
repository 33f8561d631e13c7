#!/bin/bash
# Run one gpurun call, retrying ONLY when no GPU slot or box was free
# (gpurun exit code 3: nothing ran, nothing was charged).  Any other exit
# code -- including a failed GPU step -- ends the loop at once.
#   bash scripts/gpurun_retry.sh TIMEOUT 'command'
t=$1; shift
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 90
done
exit 3
