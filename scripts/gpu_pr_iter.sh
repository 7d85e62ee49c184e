#!/bin/bash
# PageRank iteration: parity tests, then the PageRank timing for the shipped
# library and any experiment builds under csrc/build/variants.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_series_rank.py -m gpu -x -v --timeout 120 --timeout-method thread -k "pagerank or rank" > gpurun_out/gpu_pr_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_pr_tests.log; [ $rc -eq 0 ] || exit $rc
PKG=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd
: > gpurun_out/pr_time.log
timeout -k 10 100 python3 -u scripts/time_pagerank.py >> gpurun_out/pr_time.log 2>&1 || exit $?
for lib in $PKG/csrc/build/variants/libanomod_*.so; do
  [ -e "$lib" ] || continue
  echo "lib $lib" >> gpurun_out/pr_time.log
  ANOMOD_LIB=$lib timeout -k 10 100 python3 -u scripts/time_pagerank.py >> gpurun_out/pr_time.log 2>&1 || exit $?
done
echo done
