#!/bin/bash
# r05 call AH: long-trace resolve claiming 1 / 2 / 4 / 8 trace groups per
# ticket atomic (ANOMOD_RES_TICKETS); LONG, two alternating rounds; then the
# long-trace parity tests on the 4-group build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5ah
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
: > gpurun_out/r5ah/tk.log
for round in 1 2; do
  for lib in main tk2 tk4 tk8; do
    if [ $lib = main ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$GRAFT_REPO_ROOT/$V/libanomod_$lib.so; fi
    timeout -k 10 200 python3 -u scripts/r05/time_legs.py 5 LONG >> gpurun_out/r5ah/tk.log 2>&1 || exit 1
  done
done
export ANOMOD_LIB=$GRAFT_REPO_ROOT/$V/libanomod_tk4.so
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_edge.py tests/test_long_traces.py -m gpu -x -v \
  --timeout 120 --timeout-method thread -k "long" > gpurun_out/r5ah/tests.log 2>&1 || exit 2
echo done
