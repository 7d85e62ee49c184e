#!/bin/bash
# r05 call W: long-trace sets with ids staged as u32 planes and low words
# scanned (ANOMOD_SPLIT_LONG, chunk.h find_parent_split) at several widths;
# LONG leg, two alternating rounds; then the long-set parity tests on the
# 8/8 build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5w
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
: > gpurun_out/r5w/split.log
for round in 1 2; do
  for lib in main sp88 sp124 sp164 sp168 sp204; do
    if [ $lib = main ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$GRAFT_REPO_ROOT/$V/libanomod_$lib.so; fi
    timeout -k 10 200 python3 -u scripts/r05/time_legs.py 4 LONG >> gpurun_out/r5w/split.log 2>&1 || exit 1
  done
done
export ANOMOD_LIB=$GRAFT_REPO_ROOT/$V/libanomod_sp88.so
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_edge.py tests/test_long_traces.py -m gpu -x -v \
  --timeout 120 --timeout-method thread -k "long or alias" > gpurun_out/r5w/tests.log 2>&1 || exit 2
echo done
