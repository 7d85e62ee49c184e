#!/bin/bash
# r05 call C: edge / group / series tests after the first-call probe and the
# join default; first-call A/B; bench legs (upload, PageRank K = 8 / 16,
# ungrouped with its all-core CPU baseline).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/r5c
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_edge.py tests/test_gpu_group.py tests/test_gpu_series_rank.py tests/test_gpu_e2e_sn.py tests/test_gpu_e2e_tt.py -x -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 240 python3 -u scripts/r05/time_form_ab.py 27 2 SN > $O/form_sn.log 2>&1 || exit 3
timeout -k 10 240 python3 -u scripts/r05/time_form_ab.py 27 2 SN 1 > $O/form_sn_shuf.log 2>&1 || exit 4
timeout -k 10 240 python3 -u scripts/r05/time_form_ab.py 25 2 TT > $O/form_tt.log 2>&1 || exit 5
timeout -k 10 400 python3 -u bench.py --legs long_traces,pagerank,ungrouped --steps 3 --warmup 1 --no-cpu-baseline --leg-cpu-seconds 6 > $O/bench_lpu.log 2>&1 || exit 6
echo done
