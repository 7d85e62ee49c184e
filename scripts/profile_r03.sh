#!/bin/bash
# The bench process itself under rocprofv3 (kernel trace + stats), so the
# headline kernel's rocprof dispatch times and the printed bench line come from
# ONE process; then separate PMC passes (HBM bytes, SQ/LDS counters) over the
# edge, trace-structure, EWMA and grouping kernels.  Every GPU step has its own
# time limit; the script stops at the first failure.
# usage (on the box): bash scripts/profile_r03.sh [OUT]
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r03prof}
mkdir -p "$OUT"
BENCH_ARGS=${BENCH_ARGS:-"--gpus 1 --steps 20 --warmup 5"}
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 -u bench.py $BENCH_ARGS > "$OUT/bench_profiled.log" 2>&1 || exit $?
[ "${PMC:-1}" = 1 ] || { echo done; exit 0; }
PMC_ARGS="--steps 2 --warmup 0 --no-cpu-baseline --legs trace_structure,ungrouped,ewma --ewma-chunks 1"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py $PMC_ARGS > "$OUT/pmc_fetch.log" 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 bench.py $PMC_ARGS > "$OUT/pmc_write.log" 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES -d "$OUT/pmc_sq" -o run --output-format csv -- python3 bench.py $PMC_ARGS > "$OUT/pmc_sq.log" 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE -d "$OUT/pmc_sq2" -o run --output-format csv -- python3 bench.py $PMC_ARGS > "$OUT/pmc_sq2.log" 2>&1 || exit $?
echo done
