#!/bin/bash
# r05 call Y: split-word scan widths for the TrainTicket-width kernel
# (ANOMOD_WFWD / ANOMOD_WBWD with ANOMOD_SPLIT_WIDE=1); TT, two rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5y
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
: > gpurun_out/r5y/tt2.log
for round in 1 2; do
  for lib in main w124 w104 w144 w126 w122 w84; do
    if [ $lib = main ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$GRAFT_REPO_ROOT/$V/libanomod_$lib.so; fi
    timeout -k 10 200 python3 -u scripts/r05/time_legs.py 4 TT >> gpurun_out/r5y/tt2.log 2>&1 || exit 1
  done
done
echo done
