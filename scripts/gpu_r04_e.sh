#!/bin/bash
# r04: group tests (2048-record level-A tiles, no trace_hash column for the
# aggregation), then bucket-kernel occupancy variants against the default.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_group.py -v --timeout 120 --timeout-method thread \
  > gpurun_out/r4e_t.log 2>&1 || exit 1
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
for v in ship m8 s3m8 a4; do
  if [ $v = ship ]; then LIB=$PWD/anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/anomod/libanomod.so; else LIB=$PWD/$V/libanomod_$v.so; fi
  ANOMOD_LIB=$LIB AB_VAR=ANOMOD_BUCKET_DEBUG AB_VALS=0 timeout -k 10 240 python3 scripts/time_env_ab.py 27 3 \
    > gpurun_out/r4e_$v.log 2>&1 || exit 2
done
for v in ship flat; do
  if [ $v = ship ]; then LIB=$PWD/anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/anomod/libanomod.so; else LIB=$PWD/$V/libanomod_$v.so; fi
  ANOMOD_LIB=$LIB timeout -k 10 200 python3 scripts/time_ppr_ring.py 4 > gpurun_out/r4e_ppr_$v.log 2>&1 || exit 3
done
