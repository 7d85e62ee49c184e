#!/bin/bash
# EWMA iteration: series parity tests, then a timing run of the bench's EWMA leg.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_series_rank.py -m gpu -x -v --timeout 120 --timeout-method thread -k "ewma or features" > gpurun_out/gpu_ewma_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_ewma_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/time_ewma.py > gpurun_out/ewma_time.log 2>&1 || exit $?
echo done
