#!/bin/bash
# Edge kernel A/B: parity tests of the shipped build, then the shipped build
# against the experiment-only builds in csrc/build/variants (ablate_edge.py)
# on TrainTicket- and SocialNetwork-width synthetic sets (2^25 traces).
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_edge.py tests/test_long_traces.py -x -q --timeout 120 --timeout-method thread > gpurun_out/edge_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/edge_tests.log; [ $rc -eq 0 ] || exit $rc
for topo in ${AB_TOPOS:-TT SN}; do
  ABL_TOPO=$topo ABL_TRACES=${ABL_TRACES:-33554432} ABL_ROUNDS=${ABL_ROUNDS:-2} \
    timeout -k 10 400 python3 -u scripts/ablate_edge.py > gpurun_out/ab_$topo.log 2>&1 || exit $?
done
echo done
