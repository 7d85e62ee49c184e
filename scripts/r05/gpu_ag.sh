#!/bin/bash
# r05 call AG: trace-structure kernel's per-call time spread (8.1 / 8.6 /
# 9.5 ms modes) against its dynamic-tail share and segment size
# (ANOMOD_TS_DYN, ANOMOD_TS_DYN_SEG); three alternating rounds of 10 calls.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5ag
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
: > gpurun_out/r5ag/ts.log
for round in 1 2 3; do
  for lib in main seg128 seg2k dyn4 dyn1; do
    if [ $lib = main ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$GRAFT_REPO_ROOT/$V/libanomod_$lib.so; fi
    timeout -k 10 200 python3 -u scripts/r05/time_legs.py 10 TS >> gpurun_out/r5ag/ts.log 2>&1 || exit 1
  done
done
echo done
