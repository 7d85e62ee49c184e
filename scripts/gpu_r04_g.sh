#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_series_rank.py -v -k "pagerank" --timeout 120 --timeout-method thread \
  > gpurun_out/r4g_ppr_t.log 2>&1 || exit 3
timeout -k 10 200 python3 scripts/time_ppr_batch.py 2 > gpurun_out/r4g_ppr_batch.log 2>&1 || exit 4
