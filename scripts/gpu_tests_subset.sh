#!/bin/bash
# Run a subset of the GPU tests: bash scripts/gpu_tests_subset.sh tests/test_x.py ...
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest "$@" -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_subset.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_subset.log; exit $rc
