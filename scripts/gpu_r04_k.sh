#!/bin/bash
# r04: small bucket kernel ablations (no gathers / no stores / no ranking), grouping time.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_group.py -q --timeout 120 --timeout-method thread \
  > gpurun_out/r4k_t.log 2>&1 || exit 1
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
for v in ship ng ns nr ngs ngsr; do
  if [ $v = ship ]; then LIB=$PWD/anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/anomod/libanomod.so; else LIB=$PWD/$V/libanomod_$v.so; fi
  ANOMOD_LIB=$LIB AB_VAR=ANOMOD_BUCKET_DEBUG AB_VALS=0 timeout -k 10 240 python3 scripts/time_env_ab.py 27 2 \
    > gpurun_out/r4k_$v.log 2>&1 || exit 2
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in ship ngsr; do
  if [ $v = ship ]; then LIB=$PWD/anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/anomod/libanomod.so; else LIB=$PWD/$V/libanomod_$v.so; fi
  ANOMOD_LIB=$LIB AB_VAR=ANOMOD_BUCKET_DEBUG AB_VALS=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4k_kt_$v -o run --output-format csv -- python3 scripts/time_env_ab.py 27 1 > gpurun_out/r4k_kt_$v.log 2>&1 || exit 3
done
