#!/bin/bash
# Submit one gpurun call; while the pool has no free box (gpurun exit code 3: nothing ran,
# nothing charged) wait and submit it again.  Any other outcome (success or a failure of the
# command itself) ends the loop: a command that ran is never resubmitted.
#   bash scripts/gpurun_wait.sh LOG TIMEOUT 'command'
LOG=$1
TO=$2
CMD=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 150
done
exit 3
