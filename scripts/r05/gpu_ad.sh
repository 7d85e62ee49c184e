#!/bin/bash
# r05 call AD: long-trace resolve occupancy — fewer lookup spans per thread
# (ANOMOD_BIG_PER) so the kernel needs fewer VGPRs and more workgroups share a
# CU, with 1 024-id windows / 256-thread workgroups; LONG, two rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5ad
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
: > gpurun_out/r5ad/res.log
for round in 1 2; do
  for lib in main bp2w1k bp4 bp2w1kt256 bp4w1kt256 bp2; do
    if [ $lib = main ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$GRAFT_REPO_ROOT/$V/libanomod_$lib.so; fi
    timeout -k 10 200 python3 -u scripts/r05/time_legs.py 4 LONG >> gpurun_out/r5ad/res.log 2>&1 || exit 1
  done
done
echo done
