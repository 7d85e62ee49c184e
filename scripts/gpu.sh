#!/bin/bash
# Run one gpurun call; if the infrastructure reports a transient failure
# (no box / box not prepared — nothing ran, nothing charged), wait and try the
# same call again, up to 6 times.  A call that ran (any rc) is never repeated.
# usage: scripts/gpu.sh TIMEOUT 'command'
T=$1; shift
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > /tmp/gpurun_last.txt 2>&1
  rc=$?
  tail -3 /tmp/gpurun_last.txt
  if grep -q "status=transient\|backing off\|stopped responding while being prepared" /tmp/gpurun_last.txt \
     && ! grep -q "status=ok" /tmp/gpurun_last.txt; then
    echo "[gpu.sh] transient infrastructure failure, retry $i in 60s"
    sleep 60
    continue
  fi
  exit $rc
done
exit 3
