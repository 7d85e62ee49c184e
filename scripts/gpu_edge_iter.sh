#!/bin/bash
# Edge kernel iteration: edge parity tests, then variant timings.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_edge.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_edge_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_edge_tests.log; [ $rc -eq 0 ] || exit $rc
ABL_TRACES=${ABL_TRACES:-33554432} timeout -k 10 300 python3 -u scripts/ablate_edge.py > gpurun_out/ablate.log 2>&1 || exit $?
echo done
