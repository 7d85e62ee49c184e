#!/bin/bash
# r05 call X: the split-word scan (u32 id planes, low words compared) for the
# TrainTicket-width kernel (ANOMOD_SPLIT_WIDE, widths 6/4, 8/4, 12/4) and the
# SN pair form (ANOMOD_SPLIT_SN) against the shipped forms; the shipped
# build's LONG (split 12/4 now); two alternating rounds; then the edge and
# long-trace parity tests on the shipped build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5x
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
: > gpurun_out/r5x/split.log
run() {
  if [ $1 = main ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$GRAFT_REPO_ROOT/$V/libanomod_$1.so; fi
  timeout -k 10 200 python3 -u scripts/r05/time_legs.py 4 $2 >> gpurun_out/r5x/split.log 2>&1
}
for round in 1 2; do
  run main TT,SN,SNshuf,LONG || exit 1
  for v in sw64 sw84 sw124; do run $v TT || exit 1; done
  run ssn SN,SNshuf || exit 1
done
unset ANOMOD_LIB
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_edge.py tests/test_long_traces.py -m gpu -x -v \
  --timeout 120 --timeout-method thread > gpurun_out/r5x/tests.log 2>&1 || exit 2
echo done
