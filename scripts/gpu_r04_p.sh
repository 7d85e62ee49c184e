#!/bin/bash
# r04: record kernel with the ticket offsets in scalar registers: long-trace tests, LONG timing + trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_long_traces.py tests/test_gpu_edge.py -q --timeout 300 --timeout-method thread \
  > gpurun_out/r4p_t.log 2>&1 || exit 1
TG_TOPO=LONG timeout -k 10 120 python3 scripts/time_edge_leg.py 23 5 > gpurun_out/r4p_long.log 2>&1 || exit 5
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4p_kt -o run --output-format csv -- python3 scripts/time_edge_leg.py 23 3 > gpurun_out/r4p_kt.log 2>&1 || exit 6
