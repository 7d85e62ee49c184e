#!/bin/bash
# r05 call AI: where the long-trace resolve's time goes — timing-only builds
# without its inserts (1), its lookups (2), both (3); LONG leg under a kernel
# trace per build (the record pass's time moves with the parents found).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5ai
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
cd /tmp && export TMPDIR=/tmp
for lib in main ra1 ra2 ra3; do
  if [ $lib = main ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$GRAFT_REPO_ROOT/$V/libanomod_$lib.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r5ai/kt_$lib -o kt --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/scripts/r05/time_legs.py 4 LONG > $GRAFT_REPO_ROOT/gpurun_out/r5ai/kt_$lib.log 2>&1 || exit 1
done
echo done
