#!/bin/bash
# Edge-kernel ablation A/B (scripts/ablate_edge.py) on several topologies:
# AB_SPEC="TT:33554432 LONG:4194304" (topology:traces pairs).
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
for spec in ${AB_SPEC:-TT:33554432 LONG:4194304}; do
  topo=${spec%%:*}; n=${spec#*:}
  ABL_TOPO=$topo ABL_TRACES=$n ABL_ROUNDS=${ABL_ROUNDS:-2} \
    timeout -k 10 400 python3 -u scripts/ablate_edge.py > gpurun_out/ab_${TAG:-x}_$topo.log 2>&1 || exit $?
done
echo done
