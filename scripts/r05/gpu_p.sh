#!/bin/bash
# r05 call P: where the TrainTicket-width kernel's time goes after the
# select-built scan — ablation builds (1 no stats, 2 no histogram, 4 no parent
# lookup, 16 stream only) on TT and SN, two rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5p
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
: > gpurun_out/r5p/abl2.log
for round in 1 2; do
  for lib in main abl1 abl2 abl4 abl16; do
    if [ $lib = main ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$GRAFT_REPO_ROOT/$V/libanomod_$lib.so; fi
    timeout -k 10 200 python3 -u scripts/r05/time_legs.py 5 TT,LONG >> gpurun_out/r5p/abl2.log 2>&1 || exit 1
  done
done
echo done
