#!/bin/bash
# r05 call D: kernel trace of a cold (form-probing) first aggregation; request
# sizes (32 / 64 / 128 B) and DRAM-bound requests of the calibration patterns.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=$GRAFT_REPO_ROOT/gpurun_out/r5d
mkdir -p $O
export TMPDIR=/tmp
cd /tmp || exit 9
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/scripts/r05/time_form_ab.py 25 1 SN 1 > $O/kt.log 2>&1 || exit 1
find $O/kt -name "run_kernel_trace.csv" | head -1 | xargs -I{} cp {} $O/cold_trace.csv
rm -rf $O/kt
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d $O/c1 -o run --output-format csv -- \
  $GRAFT_REPO_ROOT/scripts/calib/fetch_calib 8 > $O/c1.log 2>&1 || exit 2
find $O/c1 -name "*counter_collection.csv" | head -1 | xargs -I{} cp {} $O/calib_reqsize.csv
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum -d $O/c2 -o run --output-format csv -- \
  $GRAFT_REPO_ROOT/scripts/calib/fetch_calib 8 > $O/c2.log 2>&1 || exit 3
find $O/c2 -name "*counter_collection.csv" | head -1 | xargs -I{} cp {} $O/calib_dram.csv
rm -rf $O/c1 $O/c2
echo done
