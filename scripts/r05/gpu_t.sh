#!/bin/bash
# r05 call T: trace-structure kernel with the select-built parent scan
# (ANOMOD_SEL_TS=1) against the mask form, three alternating rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5t
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
: > gpurun_out/r5t/ts.log
for round in 1 2 3; do
  for lib in main ts1; do
    if [ $lib = main ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$GRAFT_REPO_ROOT/$V/libanomod_$lib.so; fi
    timeout -k 10 200 python3 -u scripts/r05/time_legs.py 10 TS >> gpurun_out/r5t/ts.log 2>&1 || exit 1
  done
done
echo done
