#!/bin/bash
# r05 call AF: level-A record stores nontemporal (ANOMOD_BK_ABL=4 build of
# bucket.hip) against the shipped stores on the ungrouped leg; three
# alternating rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5af
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
: > gpurun_out/r5af/ug.log
for round in 1 2 3; do
  for lib in main ntA; do
    if [ $lib = main ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$GRAFT_REPO_ROOT/$V/libanomod_$lib.so; fi
    timeout -k 10 240 python3 -u scripts/r05/time_ungrouped.py 4 >> gpurun_out/r5af/ug.log 2>&1 || exit 1
  done
done
echo done
