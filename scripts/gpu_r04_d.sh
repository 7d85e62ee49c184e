#!/bin/bash
# r04: PageRank tests (persistent batch) + batch timing; group tests under the
# new defaults (one workgroup per bucket, unfused), then bucket-kernel /
# level-A tile-size variants (sper3: 1536-span small buckets, aper2:
# 2048-record level-A tiles at 2 workgroups per CU).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_series_rank.py -v -k "pagerank" --timeout 120 --timeout-method thread \
  > gpurun_out/r4d_ppr_t.log 2>&1 || exit 3
timeout -k 10 200 python3 scripts/time_ppr_batch.py 2 > gpurun_out/r4d_ppr_batch.log 2>&1 || exit 4
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_group.py -v --timeout 120 --timeout-method thread \
  > gpurun_out/r4d_t.log 2>&1 || exit 1
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
for v in ship sper3 aper2 both; do
  if [ $v = ship ]; then LIB=$PWD/anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/anomod/libanomod.so; else LIB=$PWD/$V/libanomod_$v.so; fi
  ANOMOD_LIB=$LIB AB_VAR=ANOMOD_BUCKET_DEBUG AB_VALS=0,1 timeout -k 10 240 python3 scripts/time_env_ab.py 27 2 \
    > gpurun_out/r4d_$v.log 2>&1 || exit 2
done
for v in ship bm128 bm64; do
  if [ $v = ship ]; then LIB=$PWD/anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/anomod/libanomod.so; else LIB=$PWD/$V/libanomod_$v.so; fi
  ANOMOD_LIB=$LIB TG_TOPO=LONG timeout -k 10 120 python3 scripts/time_edge_leg.py 23 5 >> gpurun_out/r4d_long.log 2>&1 || exit 5
done
