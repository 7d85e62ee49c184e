#!/bin/bash
# r05 call AB: trace-structure kernel with the split-word scan
# (ANOMOD_SPLIT_TS, widths 12/4, 6/4, 8/4) against the mask form; three
# alternating rounds of 8 calls; then the trace-structure parity tests on the
# 12/4 build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5ab
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
: > gpurun_out/r5ab/ts.log
for round in 1 2 3; do
  for lib in main ts124 ts64 ts84; do
    if [ $lib = main ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$GRAFT_REPO_ROOT/$V/libanomod_$lib.so; fi
    timeout -k 10 200 python3 -u scripts/r05/time_legs.py 8 TS >> gpurun_out/r5ab/ts.log 2>&1 || exit 1
  done
done
export ANOMOD_LIB=$GRAFT_REPO_ROOT/$V/libanomod_ts124.so
timeout -k 10 300 python3 -u -m pytest tests/test_trace_structure.py tests/test_long_traces.py -m gpu -x -v \
  --timeout 120 --timeout-method thread > gpurun_out/r5ab/tests.log 2>&1 || exit 2
echo done
