#!/bin/bash
# Trace-structure iteration: parity tests, then kernel timing.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_trace_structure.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_ts_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_ts_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u scripts/time_trace_struct.py > gpurun_out/ts_time.log 2>&1 || exit $?
echo done
