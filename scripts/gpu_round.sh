#!/bin/bash
# Full GPU check: parity tests, bench, rocprofv3 kernel-trace stats, PMC passes.
# Every GPU step has its own time limit; the script stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
[ "${SKIP_PROF:-0}" = 1 ] && exit 0
OUT=gpurun_out/prof
# rocprofv3 --kernel-trace crashes at process exit after any cooperative launch
# (scripts/coop_exit_probe.py): profiled runs take the per-launch PageRank path.
export ANOMOD_PPR_MODE=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_trace.log 2>&1 || exit $?
PMC_ARGS="--steps 2 --warmup 0 --no-cpu-baseline --no-extras"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py $PMC_ARGS > $OUT/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py $PMC_ARGS > $OUT/pmc_write.log 2>&1 || exit $?
echo done
