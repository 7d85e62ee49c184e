#!/bin/bash
# r05 call AA: long traces recorded inside the walk (list + resolve ahead of
# it) against the separate record pass (ANOMOD_BIG_FIRST=0), same process
# per round; LONG and SN; then the long-trace / edge parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5aa
: > gpurun_out/r5aa/big.log
for round in 1 2; do
  for bf in 1 0; do
    echo "== ANOMOD_BIG_FIRST=$bf" >> gpurun_out/r5aa/big.log
    ANOMOD_BIG_FIRST=$bf timeout -k 10 200 python3 -u scripts/r05/time_legs.py 4 LONG,SN >> gpurun_out/r5aa/big.log 2>&1 || exit 1
  done
done
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_edge.py tests/test_long_traces.py tests/test_gpu_e2e_sn.py -m gpu -x -v \
  --timeout 120 --timeout-method thread > gpurun_out/r5aa/tests.log 2>&1 || exit 2
echo done
