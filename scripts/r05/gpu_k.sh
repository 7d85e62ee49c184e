#!/bin/bash
# r05 call K: long-trace resolve geometry (workgroup size, window) on the
# LONG leg, every build twice, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5k
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
: > gpurun_out/r5k/res.log
for round in 1 2; do
  for lib in main t256w1024 t256w2048 t256w2048m4 t256w512 t512w1024; do
    if [ $lib = main ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$GRAFT_REPO_ROOT/$V/libanomod_$lib.so; fi
    timeout -k 10 120 python3 -u scripts/r05/time_long.py 23 4 >> gpurun_out/r5k/res.log 2>&1 || exit 1
  done
done
echo done
