#!/bin/bash
# r04: long-trace resolve variants (traces per ticket 8, 4096-id windows) on LONG.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
for v in ship g8 w4k g8w4k ship; do
  if [ $v = ship ]; then LIB=$PWD/anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/anomod/libanomod.so; else LIB=$PWD/$V/libanomod_$v.so; fi
  ANOMOD_LIB=$LIB TG_TOPO=LONG timeout -k 10 120 python3 scripts/time_edge_leg.py 23 5 >> gpurun_out/r4i_long.log 2>&1 || exit 5
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4i_kt -o run --output-format csv -- python3 scripts/time_edge_leg.py 23 3 > gpurun_out/r4i_kt.log 2>&1 || exit 6
