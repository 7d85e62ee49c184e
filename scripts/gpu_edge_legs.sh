#!/bin/bash
# Edge / trace-structure change: their GPU tests, then the bench's span legs
# (no PageRank / EWMA / config-2 legs, no CPU baseline).
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-e}
timeout -k 10 400 python -u -m pytest tests/test_gpu_edge.py tests/test_trace_structure.py tests/test_long_traces.py tests/test_gpu_group.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/edge_tests_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/edge_tests_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --legs ${LEGS:-general_scan,trace_structure,in_trace_shuffled,tt_width,long_traces} > gpurun_out/bench_$T.log 2>&1 || exit $?
echo done
