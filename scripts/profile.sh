#!/bin/bash
# rocprofv3 kernel-trace stats + separate PMC passes for the bench workload.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
OUT=gpurun_out/prof
# rocprofv3 --kernel-trace crashes at process exit after any cooperative launch
# (scripts/coop_exit_probe.py): profiled runs take the per-launch PageRank path.
export ANOMOD_PPR_MODE=1
mkdir -p $OUT
BENCH_ARGS=${BENCH_ARGS:-"--steps 5 --warmup 1 --no-cpu-baseline"}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $BENCH_ARGS > $OUT/bench_trace.log 2>&1 || exit $?
PMC_ARGS="--steps 2 --warmup 0 --no-cpu-baseline --no-extras"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py $PMC_ARGS > $OUT/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py $PMC_ARGS > $OUT/pmc_write.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES -d $OUT/pmc_sq -o run --output-format csv -- python3 bench.py $PMC_ARGS > $OUT/pmc_sq.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE -d $OUT/pmc_sq2 -o run --output-format csv -- python3 bench.py $PMC_ARGS > $OUT/pmc_sq2.log 2>&1 || exit $?
echo done
