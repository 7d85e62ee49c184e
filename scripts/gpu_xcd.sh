#!/bin/bash
# Order-hint validation (edge tests + legs) and the XCD tile-order A/B.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u scripts/time_env_ab.py 25 3 > gpurun_out/xcd25.log 2>&1 || exit $?
AB_VALS=0,3,1,2,7 timeout -k 10 300 python3 -u scripts/time_env_ab.py 27 2 > gpurun_out/xcd27.log 2>&1 || exit $?
LEGS=in_trace_shuffled,ungrouped,trace_structure TAG=o1 bash scripts/gpu_edge_legs.sh
