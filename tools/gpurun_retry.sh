#!/bin/bash
# Submit one gpurun call, re-submitting ONLY while the pool reports that no box/slot was free or
# the box was lost before the command ran (status=transient, nothing charged).  Any run that
# reached the box -- pass or fail -- ends the loop.  Usage:
#   tools/gpurun_retry.sh LOG TIMEOUT 'command'      (at most 12 attempts, 4 min apart)
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$LOG"; then
    echo "attempt $i: transient, retrying" >> "$LOG.retries"
    sleep 240
    continue
  fi
  exit $rc
done
exit 3
