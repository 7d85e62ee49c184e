#!/bin/bash
# r05 call O: parity of the select-built parent scan (TT width and long-trace
# sets): the edge, long-trace, trace-structure and TrainTicket GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5o
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_edge.py tests/test_long_traces.py \
  tests/test_trace_structure.py tests/test_gpu_e2e_tt.py tests/test_gpu_group.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/r5o/tests.log 2>&1 || exit 1
echo done
