#!/bin/bash
# gpurun, re-submitted while the pool has no free box (exit 3: nothing ran,
# nothing charged) or the box was lost while being prepared (transient: the
# service's own back-off, "retry in Ns", is waited out); any other outcome --
# including a failing command -- is returned as is.
# usage: gpurun_wait.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; shift 2
rc=3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$LOG"; then
    w=$(grep -o "retry in [0-9]*s" "$LOG" | grep -o "[0-9]*" | tail -1)
    sleep $(( ${w:-150} + 15 ))
    continue
  fi
  exit $rc
done
exit $rc
