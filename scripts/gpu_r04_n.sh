#!/bin/bash
# r04: per-chunk id hash for long-trace sets (edge tests first), then
# LONG / SN / TT timings: shipped (4 sum replicas, hash above 48-span traces),
# 8 replicas (no room for the hash), no hash, hash thresholds 24 / 96.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_edge.py tests/test_long_traces.py tests/test_gpu_group.py -q --timeout 300 --timeout-method thread \
  > gpurun_out/r4n_t.log 2>&1 || exit 1
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
for topo in LONG SN TT; do
  lg=27; [ $topo = LONG ] && lg=23
  for v in ship rep8 nohash hm24 hm96; do
    [ $topo != LONG ] && [ $v != ship ] && [ $v != rep8 ] && continue
    if [ $v = ship ]; then LIB=$PWD/anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/anomod/libanomod.so; else LIB=$PWD/$V/libanomod_$v.so; fi
    ANOMOD_LIB=$LIB TG_TOPO=$topo timeout -k 10 120 python3 scripts/time_edge_leg.py $lg 5 >> gpurun_out/r4n_legs.log 2>&1 || exit 5
  done
done
