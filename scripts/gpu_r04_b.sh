#!/bin/bash
# r04: PageRank ring tests + A/B, then the grouping PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_series_rank.py tests/test_gpu_host_comm.py -v -k "pagerank or two_ranks" --timeout 120 --timeout-method thread \
  > gpurun_out/r4_ppr_t.log 2>&1 || exit 1
timeout -k 10 200 python3 scripts/time_ppr_ring.py 5 > gpurun_out/r4_ppr_ring.log 2>&1 || exit 2
LG=26 ./scripts/gpu_r04_pmc_ug.sh || exit 3
