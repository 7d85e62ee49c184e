#!/bin/bash
# One box, several steps: GPU tests, the full bench, then the edge ablation
# builds per topology.  Each step has its own time limit; stop at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-g}
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 ${BENCH_EXTRA:-} > gpurun_out/bench_$T.log 2>&1 || exit $?
[ "${ABL:-1}" = 1 ] || exit 0
for spec in ${AB_SPEC:-SN:33554432 TT:33554432 LONG:4194304}; do
  topo=${spec%%:*}; n=${spec#*:}
  ABL_TOPO=$topo ABL_TRACES=$n ABL_ROUNDS=1 \
    timeout -k 10 300 python3 -u scripts/ablate_edge.py > gpurun_out/ab_${T}_$topo.log 2>&1 || exit $?
done
echo done
