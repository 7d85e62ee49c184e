#!/bin/bash
# EWMA kernel variants (experiment builds under csrc/build/variants) timed on the bench shape.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
echo "main" > gpurun_out/ewma_sweep.log
timeout -k 10 120 python3 -u scripts/time_ewma.py >> gpurun_out/ewma_sweep.log 2>&1 || exit $?
for lib in $V/libanomod_ewma*.so; do
  echo "$lib" >> gpurun_out/ewma_sweep.log
  ANOMOD_LIB=$lib timeout -k 10 120 python3 -u scripts/time_ewma.py >> gpurun_out/ewma_sweep.log 2>&1 || exit $?
done
