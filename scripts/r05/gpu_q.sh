#!/bin/bash
# r05 call Q: long-trace record kernel with the next block's loads issued
# before the current block's records (ANOMOD_REC_PIPE), and the spans per
# thread per block (ANOMOD_REC_PER); LONG leg, two alternating rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5q
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
: > gpurun_out/r5q/rec.log
for round in 1 2; do
  for lib in main rp0 rp2 rp8; do
    if [ $lib = main ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$GRAFT_REPO_ROOT/$V/libanomod_$lib.so; fi
    timeout -k 10 200 python3 -u scripts/r05/time_legs.py 5 LONG >> gpurun_out/r5q/rec.log 2>&1 || exit 1
  done
done
unset ANOMOD_LIB
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r5q/kt -o kt --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/scripts/r05/time_legs.py 5 LONG > $GRAFT_REPO_ROOT/gpurun_out/r5q/kt.log 2>&1 || exit 2
echo done
