#!/bin/bash
# r05 call AE: the split-word scan's match search as a min over
# (miss << 5 | slot) keys (ANOMOD_SPLIT_ARITH=1: xor / min / shift-or and
# pairwise min trees, no compare-select chain) against the select chain; TT
# and LONG, two alternating rounds; then the alias / long parity tests on it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5ae
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
: > gpurun_out/r5ae/arith.log
for round in 1 2; do
  for lib in main arith; do
    if [ $lib = main ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$GRAFT_REPO_ROOT/$V/libanomod_$lib.so; fi
    timeout -k 10 200 python3 -u scripts/r05/time_legs.py 5 TT,LONG >> gpurun_out/r5ae/arith.log 2>&1 || exit 1
  done
done
export ANOMOD_LIB=$GRAFT_REPO_ROOT/$V/libanomod_arith.so
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_edge.py -m gpu -x -v --timeout 120 \
  --timeout-method thread -k "alias or long or unique" > gpurun_out/r5ae/tests.log 2>&1 || exit 2
echo done
