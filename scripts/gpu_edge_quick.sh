#!/bin/bash
# Edge parity tests, then the shipped library timed per topology
# (AB_SPEC="SN:33554432 TT:33554432 LONG:4194304"; ABL_GLOB selects variant builds).
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_edge.py tests/test_long_traces.py} -x -q --timeout 120 --timeout-method thread > gpurun_out/edge_tests_${TAG:-q}.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/edge_tests_${TAG:-q}.log; [ $rc -eq 0 ] || exit $rc
for spec in ${AB_SPEC:-SN:33554432 TT:33554432 LONG:4194304}; do
  topo=${spec%%:*}; n=${spec#*:}
  ABL_TOPO=$topo ABL_TRACES=$n ABL_ROUNDS=${ABL_ROUNDS:-1} ABL_GLOB=${ABL_GLOB:-none} \
    timeout -k 10 300 python3 -u scripts/ablate_edge.py > gpurun_out/ab_${TAG:-q}_$topo.log 2>&1 || exit $?
done
echo done
