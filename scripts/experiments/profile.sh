#!/bin/bash
# Bench, then rocprofv3 kernel-trace stats of the same bench command, then
# separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) over the headline edge
# kernel + trace-structure + one EWMA chunk, all on the same box.
# Every GPU step has its own time limit; the script stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
BENCH_ARGS=${BENCH_ARGS:-"--steps 10 --warmup 2"}
timeout -k 10 300 python3 -u bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $BENCH_ARGS --no-cpu-baseline > $OUT/bench_trace.log 2>&1 || exit $?
PMC_ARGS="--steps 2 --warmup 0 --no-cpu-baseline --legs trace_structure,ewma --ewma-chunks 1"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py $PMC_ARGS > $OUT/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py $PMC_ARGS > $OUT/pmc_write.log 2>&1 || exit $?
if [ "${SQ_PASSES:-1}" = 1 ]; then
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES -d $OUT/pmc_sq -o run --output-format csv -- python3 bench.py $PMC_ARGS > $OUT/pmc_sq.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE -d $OUT/pmc_sq2 -o run --output-format csv -- python3 bench.py $PMC_ARGS > $OUT/pmc_sq2.log 2>&1 || exit $?
fi
echo done
