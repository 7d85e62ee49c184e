#!/bin/bash
# r04: long-trace record kernel with 4 / 8 / 16 listed spans per thread in flight (LONG).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
for v in ship rp8 rp16 ship; do
  if [ $v = ship ]; then LIB=$PWD/anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/anomod/libanomod.so; else LIB=$PWD/$V/libanomod_$v.so; fi
  ANOMOD_LIB=$LIB TG_TOPO=LONG timeout -k 10 120 python3 scripts/time_edge_leg.py 23 5 >> gpurun_out/r4o_long.log 2>&1 || exit 5
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in rp8 rp16; do
  ANOMOD_LIB=$PWD/$V/libanomod_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4o_kt_$v -o run --output-format csv -- python3 scripts/time_edge_leg.py 23 3 > gpurun_out/r4o_kt_$v.log 2>&1 || exit 6
done
