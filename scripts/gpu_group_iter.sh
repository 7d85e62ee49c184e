#!/bin/bash
# Grouping iteration: the group tests, then the bucket-vs-LSD timing.
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-g}
timeout -k 10 300 python -u -m pytest tests/test_gpu_group.py -x -v --timeout 120 --timeout-method thread > gpurun_out/grp_tests_$T.log 2>&1 || exit $?
timeout -k 10 300 python3 -u scripts/time_group_paths.py ${LG:-25} 3 ${AVGS:-1400} > gpurun_out/grp_time_$T.log 2>&1 || exit $?
[ -n "$FULL" ] || exit 0
timeout -k 10 300 python3 -u scripts/time_group_paths.py 27 2 ${AVGS:-1400} > gpurun_out/grp_time27_$T.log 2>&1 || exit $?
TG_TOPO=LONG timeout -k 10 300 python3 -u scripts/time_group_paths.py 22 2 ${AVGS:-1400} > gpurun_out/grp_timeLONG_$T.log 2>&1 || exit $?
TG_TOPO=TT timeout -k 10 300 python3 -u scripts/time_group_paths.py 25 2 ${AVGS:-1400} > gpurun_out/grp_timeTT_$T.log 2>&1 || exit $?
