#!/bin/bash
# r05 call V: cooperative completion of the parent lookups (after N per-lane
# scan steps the wave finishes the rest with 64-id ballot scans,
# ANOMOD_COOP_STEPS) on LONG, TT and SN; two alternating rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5v
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
: > gpurun_out/r5v/coop.log
for round in 1 2; do
  for lib in main c2 c3 c5; do
    if [ $lib = main ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$GRAFT_REPO_ROOT/$V/libanomod_$lib.so; fi
    timeout -k 10 200 python3 -u scripts/r05/time_legs.py 4 LONG,TT,SN >> gpurun_out/r5v/coop.log 2>&1 || exit 1
  done
done
echo done
