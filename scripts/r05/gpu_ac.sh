#!/bin/bash
# r05 call AC: the SN pair form with the split-word scan at wider steps
# (ANOMOD_SPLIT_SN=1, 12/4, 10/4, 8/4) on SN and in-trace-shuffled SN; three
# alternating rounds of 6 calls.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5ac
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
: > gpurun_out/r5ac/sn.log
for round in 1 2 3; do
  for lib in main ssn124 ssn104 ssn84; do
    if [ $lib = main ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$GRAFT_REPO_ROOT/$V/libanomod_$lib.so; fi
    timeout -k 10 200 python3 -u scripts/r05/time_legs.py 6 SN,SNshuf >> gpurun_out/r5ac/sn.log 2>&1 || exit 1
  done
done
echo done
