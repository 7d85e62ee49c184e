#!/bin/bash
# r05 call AJ: the long-trace resolve's inserts store a unique-id slot's
# position plainly (ANOMOD_RES_UNI_STORE=1, shipped candidate) against
# atomicMin (=0); LONG under a kernel trace per build, two rounds; then the
# long-trace parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5aj
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
cd /tmp && export TMPDIR=/tmp
for round in 1 2; do
  for lib in main us0; do
    if [ $lib = main ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$GRAFT_REPO_ROOT/$V/libanomod_$lib.so; fi
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r5aj/kt_${lib}_$round -o kt --output-format csv -- \
      python3 $GRAFT_REPO_ROOT/scripts/r05/time_legs.py 4 LONG > $GRAFT_REPO_ROOT/gpurun_out/r5aj/kt_${lib}_$round.log 2>&1 || exit 1
  done
done
cd $GRAFT_REPO_ROOT && unset ANOMOD_LIB
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_edge.py tests/test_long_traces.py -m gpu -x -v \
  --timeout 120 --timeout-method thread > gpurun_out/r5aj/tests.log 2>&1 || exit 2
echo done
