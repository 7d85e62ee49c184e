#!/bin/bash
# Runs one gpurun call; when the pool had no slot or box, or the box failed
# while being prepared (nothing ran, nothing charged: "retry in a few
# minutes" / status=transient), waits and asks again, at most 12 times.  A call that ran is never repeated.
# usage: scripts/gpurun_retry.sh OUTFILE 'command'
out=$1; shift
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout ${GPURUN_TIMEOUT:-1200} -- "$@" > "$out" 2>&1
  rc=$?
  if grep -Eq "retry in|status=transient" "$out" && grep -Eq "charged=(0\.0s|None)" "$out"; then
    sleep 120
    continue
  fi
  exit $rc
done
exit 3
