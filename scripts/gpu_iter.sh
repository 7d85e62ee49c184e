#!/bin/bash
# GPU iteration: parity tests, then ablation timings, then a short bench.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/ablate_edge.py > gpurun_out/ablate.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 5 > gpurun_out/bench.log 2>&1
echo "bench rc=$?" >> gpurun_out/bench.log
