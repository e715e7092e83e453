#!/bin/bash
# gpurun, re-submitted while the pool has no free box (exit 3: nothing ran,
# nothing charged) or the box was lost while being prepared (transient); any
# other outcome -- including a failing command -- is returned as is.
# usage: gpurun_wait.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; shift 2
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$LOG"; then sleep 150; continue; fi
  exit $rc
done
exit $rc
