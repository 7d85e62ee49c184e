#!/bin/bash
# r04: grouping tests, bucket-kernel pipelining A/B (shipped: MINB 2; variant
# pipe4: 4 waves per SIMD with spills), fused and unfused; PPR ring tests + A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_group.py tests/test_gpu_series_rank.py tests/test_gpu_host_comm.py -v -k "group or ungrouped or pagerank or two_ranks" --timeout 120 --timeout-method thread \
  > gpurun_out/r4c_t.log 2>&1 || exit 1
for fz in 0 1; do
  ANOMOD_UNGROUPED_FUSED=$fz AB_VAR=ANOMOD_BK_PIPE AB_VALS=1,0 timeout -k 10 240 python3 scripts/time_env_ab.py 27 2 \
    > gpurun_out/r4c_pipe_f$fz.log 2>&1 || exit 2
done
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
ANOMOD_LIB=$PWD/$V/libanomod_pipe4.so AB_VAR=ANOMOD_UNGROUPED_FUSED AB_VALS=0,1 timeout -k 10 240 python3 scripts/time_env_ab.py 27 2 \
  > gpurun_out/r4c_pipe4.log 2>&1 || exit 3
timeout -k 10 200 python3 scripts/time_ppr_ring.py 5 > gpurun_out/r4c_ppr_ring.log 2>&1 || exit 4
