#!/bin/bash
# GPU tests + a bench run of selected legs.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_${TAG:-b}.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_${TAG:-b}.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline ${LEGS:+--legs $LEGS} > gpurun_out/bench_${TAG:-b}.log 2>&1
