#!/bin/bash
# r05 call A: grouping/join tests, new join A/B (fast vs stable level B; 8 vs 6
# waves per SIMD for the join), kernel trace of the ungrouped leg at 2^27 SN
# traces, FETCH_SIZE calibration of gathers / narrow streams.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5a
O=gpurun_out/r5a
timeout -k 10 420 python3 -u -m pytest tests/test_gpu_group.py -x -v --timeout 120 --timeout-method thread \
  > $O/grp_tests.log 2>&1 || exit 1
AB_VAR=ANOMOD_BK_STABLE_B AB_VALS=0,1 timeout -k 10 240 python3 -u scripts/time_env_ab.py 27 3 \
  > $O/ab_stableb.log 2>&1 || exit 2
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
AB_VAR=NONE AB_VALS=x ANOMOD_LIB=$PWD/$V/libanomod_jm6.so timeout -k 10 240 python3 -u scripts/time_env_ab.py 27 3 \
  > $O/ab_jm6.log 2>&1 || exit 3
timeout -k 10 120 ./scripts/calib/fetch_calib 8 > $O/calib_time.log 2>&1 || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$GRAFT_REPO_ROOT/$O/calib_pmc" -o run --output-format csv -- \
  "$GRAFT_REPO_ROOT/scripts/calib/fetch_calib" 8 > "$GRAFT_REPO_ROOT/$O/calib_pmc.log" 2>&1 || exit 5
find "$GRAFT_REPO_ROOT/$O/calib_pmc" -name "*counter_collection.csv" | head -1 | xargs -I{} cp {} "$GRAFT_REPO_ROOT/$O/calib_fetch.csv"
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$GRAFT_REPO_ROOT/$O/calib_pmc2" -o run --output-format csv -- \
  "$GRAFT_REPO_ROOT/scripts/calib/fetch_calib" 8 > "$GRAFT_REPO_ROOT/$O/calib_pmc2.log" 2>&1 || exit 6
find "$GRAFT_REPO_ROOT/$O/calib_pmc2" -name "*counter_collection.csv" | head -1 | xargs -I{} cp {} "$GRAFT_REPO_ROOT/$O/calib_hitmiss.csv"
rm -rf "$GRAFT_REPO_ROOT/$O/calib_pmc" "$GRAFT_REPO_ROOT/$O/calib_pmc2"
AB_VAR=NONE AB_VALS=x timeout -k 10 300 rocprofv3 --kernel-trace --stats \
  -d "$GRAFT_REPO_ROOT/$O/prof_ug" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/scripts/time_env_ab.py" 27 1 > "$GRAFT_REPO_ROOT/$O/prof_ug.log" 2>&1 || exit 7
find "$GRAFT_REPO_ROOT/$O/prof_ug" -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} "$GRAFT_REPO_ROOT/$O/kstats_ug.csv"
rm -rf "$GRAFT_REPO_ROOT/$O/prof_ug"
echo done
