#!/bin/bash
# GPU tests, then the one-process profile (scripts/profile_r03.sh).
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r03a.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_r03a.log; [ $rc -eq 0 ] || exit $rc
bash scripts/profile_r03.sh gpurun_out/r03prof
