#!/bin/bash
# Full GPU check: parity tests, then scripts/profile.sh (bench, rocprofv3
# kernel-trace stats of the same bench command, PMC passes) on the same box.
# Every GPU step has its own time limit; the script stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
if [ "${SKIP_PROF:-0}" = 1 ]; then
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1
  exit $?
fi
bash scripts/profile.sh
