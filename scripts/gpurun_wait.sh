#!/bin/bash
# gpurun with waits while the pool has no box for the call (nothing ran and
# nothing was charged); any call that ran returns at once, whatever its exit.
#   bash scripts/gpurun_wait.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; shift 2
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient\|slot(s) on this pod are busy\|no free box" "$LOG"; then
    sleep 100; continue
  fi
  exit $rc
done
exit $rc
