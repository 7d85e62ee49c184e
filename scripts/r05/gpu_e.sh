#!/bin/bash
# r05 call E: edge tests after the merged first-call probes; first-call A/B at
# 2^27 (SN, shuffled SN); kernel trace of a cold 2^27 SN first call.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=$GRAFT_REPO_ROOT/gpurun_out/r5e
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_edge.py tests/test_long_traces.py tests/test_gpu_group.py -x -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 240 python3 -u scripts/r05/time_form_ab.py 27 2 SN > $O/form_sn.log 2>&1 || exit 2
timeout -k 10 240 python3 -u scripts/r05/time_form_ab.py 27 2 SN 1 > $O/form_sn_shuf.log 2>&1 || exit 3
export TMPDIR=/tmp
cd /tmp || exit 9
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/scripts/r05/time_form_ab.py 27 1 SN > $O/kt.log 2>&1 || exit 4
find $O/kt -name "run_kernel_trace.csv" | head -1 | xargs -I{} cp {} $O/cold_trace.csv
rm -rf $O/kt
echo done
