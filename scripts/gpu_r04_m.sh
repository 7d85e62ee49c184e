#!/bin/bash
# r04: small bucket kernel with atomic slots + compare rank (variant rank1):
# group tests under it, then grouping time against the shipped stable split.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
V=$PWD/anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
ANOMOD_LIB=$V/libanomod_rank1.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_group.py -q --timeout 120 --timeout-method thread \
  > gpurun_out/r4m_t.log 2>&1 || exit 1
for v in ship rank1 ship rank1; do
  if [ $v = ship ]; then LIB=$PWD/anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/anomod/libanomod.so; else LIB=$V/libanomod_$v.so; fi
  ANOMOD_LIB=$LIB AB_VAR=ANOMOD_BUCKET_DEBUG AB_VALS=0 timeout -k 10 240 python3 scripts/time_env_ab.py 27 2 \
    >> gpurun_out/r4m_$v.log 2>&1 || exit 2
done
ANOMOD_LIB=$V/libanomod_rank1.so TG_TOPO=TT AB_VAR=ANOMOD_BUCKET_DEBUG AB_VALS=0 timeout -k 10 240 python3 scripts/time_env_ab.py 25 2 > gpurun_out/r4m_tt_rank1.log 2>&1 || exit 3
TG_TOPO=TT AB_VAR=ANOMOD_BUCKET_DEBUG AB_VALS=0 timeout -k 10 240 python3 scripts/time_env_ab.py 25 2 > gpurun_out/r4m_tt_ship.log 2>&1 || exit 4
