#!/bin/bash
# r06 profile: the bench process itself under rocprofv3 (kernel trace +
# stats: the headline kernel's dispatch times and the printed line come from
# ONE process), then PMC passes (HBM bytes; SQ / LDS counters) over a reduced
# bench that runs every leg whose kernels the summary names.  Each GPU step
# has its own time limit; the script stops at the first failure.
# usage (on the box): bash scripts/profile_r06.sh [OUT]
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
OUT=${1:-$GRAFT_REPO_ROOT/gpurun_out/r06prof}
mkdir -p "$OUT"
BENCH_ARGS=${BENCH_ARGS:-"--gpus 1 --steps 20 --warmup 5"}
if [ "${TRACE:-1}" = 1 ]; then
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
    -- python3 -u bench.py $BENCH_ARGS > "$OUT/bench_profiled.log" 2>&1 || exit $?
  find "$OUT/trace" -name "run_kernel_stats.csv" | head -1 | xargs -I{} cp {} "$OUT/kernel_stats.csv"
  find "$OUT/trace" -name "run_kernel_trace.csv" | head -1 | xargs -I{} cp {} "$OUT/kernel_trace.csv"
  rm -rf "$OUT/trace"
fi
[ "${PMC:-1}" = 1 ] || { echo done; exit 0; }
PMC_ARGS=${PMC_ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline --legs trace_structure,ungrouped,tt_width,long_traces,pagerank,ewma --ewma-chunks 1"}
i=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE" \
            "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" \
            "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $ctrs -d "$OUT/p$i" -o run --output-format csv -- \
    python3 bench.py $PMC_ARGS > "$OUT/p$i.log" 2>&1 || exit $((10+i))
  find "$OUT/p$i" -name "*counter_collection.csv" | head -1 | xargs -I{} cp {} "$OUT/p$i.csv"
  rm -rf "$OUT/p$i"
done
echo done
