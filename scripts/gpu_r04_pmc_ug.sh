#!/bin/bash
# PMC passes (HBM bytes, SQ) over the grouping kernels of the ungrouped path
# (time_env_ab.py at 2^LG SN traces, unfused), one pass per counter group.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
export TMPDIR=/tmp
LG=${LG:-26}
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4pmc_ug
mkdir -p "$OUT"
cd /tmp || exit 9
export AB_VAR=ANOMOD_UNGROUPED_FUSED AB_VALS=0
i=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE" \
            "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" \
            "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $ctrs -d "$OUT/p$i" -o run --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/scripts/time_env_ab.py" $LG 1 > "$OUT/p$i.log" 2>&1 || exit $i
  find "$OUT/p$i" -name "*counter_collection.csv" | head -1 | xargs -I{} cp {} "$OUT/p$i.csv"
  rm -rf "$OUT/p$i"
done
echo done
