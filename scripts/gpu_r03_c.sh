#!/bin/bash
# Round-3 check: every GPU test, then the default bench line.  Each step has
# its own time limit; stop at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-c}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$T.log 2>&1 || exit $?
echo done
