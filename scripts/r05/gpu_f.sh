#!/bin/bash
# r05 call F: PageRank tests (K = 16 split kernel), the PageRank bench leg;
# first call with the set read once before (first-touch check).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=$GRAFT_REPO_ROOT/gpurun_out/r5f
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_series_rank.py -x -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --legs pagerank --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_ppr.log 2>&1 || exit 2
timeout -k 10 240 python3 -u scripts/r05/time_form_ab.py 27 1 SN 0 1 > $O/form_touch.log 2>&1 || exit 3
timeout -k 10 240 python3 -u scripts/r05/time_form_ab.py 27 1 SN 0 0 > $O/form_notouch.log 2>&1 || exit 4
echo done
