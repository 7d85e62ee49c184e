#!/bin/bash
# Edge kernel: ablation/variant timings, then SQ/LDS counter passes on the
# shipped build (one GPU call).  Every GPU step has its own time limit; the
# script stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
OUT=gpurun_out/prof_edge
mkdir -p $OUT
export ABL_TRACES=${ABL_TRACES:-33554432}
timeout -k 10 400 python3 -u scripts/experiments/ablate_edge.py > $OUT/ablate.log 2>&1 || exit $?
[ "${SKIP_PMC:-0}" = 1 ] && exit 0
run() { name=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" -d $OUT/$name -o run --output-format csv -- python3 scripts/experiments/ablate_edge.py --one > $OUT/$name.log 2>&1 || exit $?; }
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES
run sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA
run grbm GRBM_GUI_ACTIVE GRBM_COUNT
echo done
