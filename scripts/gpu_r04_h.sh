#!/bin/bash
# r04: the whole GPU suite, then edge-kernel timings of the three widths.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r4h_t.log 2>&1 || exit 1
for topo in LONG SN TT; do
  lg=27; [ $topo = LONG ] && lg=23
  TG_TOPO=$topo timeout -k 10 120 python3 scripts/time_edge_leg.py $lg 4 >> gpurun_out/r4h_legs.log 2>&1 || exit 5
done
timeout -k 10 200 python3 scripts/time_ppr_batch.py 2 > gpurun_out/r4h_ppr_batch.log 2>&1 || exit 4
