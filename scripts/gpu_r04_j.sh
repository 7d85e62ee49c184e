#!/bin/bash
# r04: the SN column stream at 8/4-B vs 16-B loads per lane (stream-only builds).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
for v in ship s8 s16 s8 s16; do
  if [ $v = ship ]; then LIB=$PWD/anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/anomod/libanomod.so; else LIB=$PWD/$V/libanomod_$v.so; fi
  ANOMOD_LIB=$LIB TG_TOPO=SN timeout -k 10 120 python3 scripts/time_edge_leg.py 27 6 >> gpurun_out/r4j_stream.log 2>&1 || exit 5
done
