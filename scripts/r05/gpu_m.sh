#!/bin/bash
# r05 call M: parent scan with select-built indexes and both blocks' loads
# in one round trip (ANOMOD_BIDIR_SEL=1) against the shipped scan, every set,
# two alternating rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5m
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
: > gpurun_out/r5m/legs.log
for round in 1 2; do
  for lib in main sel1; do
    if [ $lib = main ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$GRAFT_REPO_ROOT/$V/libanomod_$lib.so; fi
    timeout -k 10 200 python3 -u scripts/r05/time_legs.py 4 >> gpurun_out/r5m/legs.log 2>&1 || exit 1
  done
done
echo done
