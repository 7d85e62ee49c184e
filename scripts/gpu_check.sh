#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1
timeout -k 10 400 python -u -m pytest tests -m "gpu and not slow" -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cpu-seconds 5 > gpurun_out/bench.log 2>&1
echo "bench rc=$?" >> gpurun_out/bench.log
exit $rc
