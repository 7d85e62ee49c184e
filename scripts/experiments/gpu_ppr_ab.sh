#!/bin/bash
# PageRank A/B: the shipped build and every csrc/build/variants/libanomod_prb*.so
# through scripts/experiments/time_pagerank.py (persistent SUB sweep inside).
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
: > gpurun_out/ppr.log
for lib in main anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants/libanomod_prb*.so; do
  echo "lib=$lib" >> gpurun_out/ppr.log
  if [ "$lib" = main ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$PWD/$lib; fi
  PPR_MODES=${PPR_MODES:-0,2} timeout -k 10 120 python -u scripts/experiments/time_pagerank.py >> gpurun_out/ppr.log 2>&1 || exit $?
done
