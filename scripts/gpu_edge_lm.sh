#!/bin/bash
# Edge kernel parity tests, then the shipped build against the experiment
# builds in csrc/build/variants on TT, SN and LONG synthetic sets.
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_edge.py tests/test_long_traces.py tests/test_gpu_e2e_tt.py -x -q --timeout 120 --timeout-method thread > gpurun_out/edge_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/edge_tests.log; [ $rc -eq 0 ] || exit $rc
for spec in ${AB_SPECS:-TT:33554432 SN:33554432 LONG:4194304}; do
  topo=${spec%%:*}; n=${spec##*:}
  ABL_TOPO=$topo ABL_TRACES=$n ABL_ROUNDS=${ABL_ROUNDS:-2} \
    timeout -k 10 400 python3 -u scripts/ablate_edge.py > gpurun_out/ab_$topo.log 2>&1 || exit $?
done
echo done
