#!/bin/bash
# LONG leg (2^23 traces) under edge_agg.hip variants (build/variants), each in
# its own process, alternating; digests must agree.  LIBS names the variants.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
for lib in ${LIBS:-ship orig ship orig}; do
  if [ "$lib" = ship ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$PWD/$V/libanomod_$lib.so; fi
  echo "== $lib $(TG_TOPO=${TOPO:-LONG} timeout -k 10 120 python3 scripts/time_edge_leg.py ${LG:-23} 5 | tail -1)" || exit 1
done
exit 0
