#!/bin/bash
# r04: cooperative completion of the parent lookups (per-lane scan steps 1 /
# 2 / 3, then the whole wave): edge tests under c1 and c2, then SN / TT / LONG timings.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
V=$PWD/anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
for v in c1 c2; do
  ANOMOD_LIB=$V/libanomod_$v.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_edge.py tests/test_long_traces.py tests/test_gpu_group.py -q --timeout 300 --timeout-method thread \
    > gpurun_out/r4r_t_$v.log 2>&1 || exit 1
done
for topo in TT SN LONG; do
  lg=27; [ $topo = LONG ] && lg=23
  for v in ship c1 c2 c3; do
    if [ $v = ship ]; then LIB=$PWD/anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/anomod/libanomod.so; else LIB=$V/libanomod_$v.so; fi
    ANOMOD_LIB=$LIB TG_TOPO=$topo timeout -k 10 120 python3 scripts/time_edge_leg.py $lg 4 >> gpurun_out/r4r_legs.log 2>&1 || exit 5
  done
done
