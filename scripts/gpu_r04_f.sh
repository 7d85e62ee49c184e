#!/bin/bash
# r04: PageRank tests + batch timing (write-through coalesced stores, pinned
# staging); bidirectional-scan widths (kFwd/kBwd) on SN / TT / LONG.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_series_rank.py -v -k "pagerank" --timeout 120 --timeout-method thread \
  > gpurun_out/r4f_ppr_t.log 2>&1 || exit 3
timeout -k 10 200 python3 scripts/time_ppr_batch.py 2 > gpurun_out/r4f_ppr_batch.log 2>&1 || exit 4
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
for topo in TT SN LONG; do
  lg=27; [ $topo = LONG ] && lg=23
  for v in ship f8b4 f6b6 f8b8 f4b4 f4b2; do
    if [ $v = ship ]; then LIB=$PWD/anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/anomod/libanomod.so; else LIB=$PWD/$V/libanomod_$v.so; fi
    ANOMOD_LIB=$LIB TG_TOPO=$topo timeout -k 10 120 python3 scripts/time_edge_leg.py $lg 4 >> gpurun_out/r4f_scan.log 2>&1 || exit 5
  done
done
