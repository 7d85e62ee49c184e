#!/bin/bash
# r04: persistent PageRank workgroup size (256-row blocks per workgroup 1 / 2 / 4) with the ring.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for sub in 1 2 4 1; do
  ANOMOD_PPR_SUB=$sub timeout -k 10 200 python3 scripts/time_ppr_ring.py 3 > gpurun_out/r4l_sub$sub.log 2>&1 || exit 3
done
