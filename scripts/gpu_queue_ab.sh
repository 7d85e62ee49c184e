#!/bin/bash
# Per-lane lookup queue (edge_agg.hip ANOMOD_QUEUE): shipped (1: long-trace
# sets) vs q0 (off) vs q3 (also the default unique-id scan), LONG 2^23 / TT
# 2^25 / SN 2^27, each in its own process; the digests must agree.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
for leg in "LONG 23" "TT 25" "SN 27"; do
  set -- $leg
  for lib in ${LIBS:-ship q0 q3 ship q0 q3}; do
    if [ "$lib" = ship ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$PWD/$V/libanomod_$lib.so; fi
    echo "== $1 $lib $(TG_TOPO=$1 timeout -k 10 120 python3 scripts/time_edge_leg.py $2 5 | tail -1)" || exit 1
  done
done
exit 0
