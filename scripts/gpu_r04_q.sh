#!/bin/bash
# r04: TrainTicket-width ablations (no stats / no histogram / no parent lookup / stream only).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
for topo in TT LONG; do
  lg=27; [ $topo = LONG ] && lg=23
  for v in ship a1 a2 a4 a16; do
    if [ $v = ship ]; then LIB=$PWD/anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/anomod/libanomod.so; else LIB=$PWD/$V/libanomod_$v.so; fi
    ANOMOD_LIB=$LIB TG_TOPO=$topo timeout -k 10 120 python3 scripts/time_edge_leg.py $lg 4 >> gpurun_out/r4q_abl.log 2>&1 || exit 5
  done
done
