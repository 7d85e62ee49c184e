#!/bin/bash
# LDS-pipe counters of the edge kernel (two PMC passes, one run each) on the
# ablation script's workload; summaries land in gpurun_out/lds_pmc*/.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
OUT=gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INSTS_LDS SQ_BUSY_CU_CYCLES -d $OUT/lds_pmc1 -o run --output-format csv -- python3 scripts/ablate_edge.py --one > $OUT/lds_pmc1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_ATOMIC SQ_INSTS_LDS_STORE SQ_INSTS_LDS_LOAD_BANDWIDTH SQ_INSTS_LDS_ATOMIC_BANDWIDTH SQ_INSTS_LDS_STORE_BANDWIDTH SQ_WAIT_INST_LDS SQ_WAVE_CYCLES -d $OUT/lds_pmc2 -o run --output-format csv -- python3 scripts/ablate_edge.py --one > $OUT/lds_pmc2.log 2>&1 || exit $?
echo done
