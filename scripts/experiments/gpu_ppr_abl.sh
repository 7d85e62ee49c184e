#!/bin/bash
# PageRank persistent-solve ablations (timing only): shipped / no gathers /
# no grid barrier / neither, N = 1e5 config-5 graph.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
for lib in ship pabl1 pabl2 pabl3; do
  if [ "$lib" = ship ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$PWD/$V/libanomod_$lib.so; fi
  echo "== $lib"
  PPR_MODES=2 PPR_SUBS=1 timeout -k 10 120 python3 scripts/experiments/time_pagerank.py || exit 1
done
