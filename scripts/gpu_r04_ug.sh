#!/bin/bash
# r04: ungrouped path — grouping tests, fused vs unfused and XCD-order A/B at
# 2^27 SN traces, then a kernel trace of the same run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_group.py -v --timeout 120 --timeout-method thread \
  > gpurun_out/r4_grp_t.log 2>&1 || exit 1
AB_VAR=ANOMOD_UNGROUPED_FUSED AB_VALS=1,0 timeout -k 10 240 python3 scripts/time_env_ab.py 27 3 \
  > gpurun_out/r4_ab_fused.log 2>&1 || exit 2
AB_VAR=ANOMOD_BK_XCD AB_VALS=3,7 timeout -k 10 240 python3 scripts/time_env_ab.py 27 3 \
  > gpurun_out/r4_ab_xcd.log 2>&1 || exit 3
cd /tmp && export TMPDIR=/tmp
AB_VAR=ANOMOD_UNGROUPED_FUSED AB_VALS=1,0 timeout -k 10 300 rocprofv3 --kernel-trace --stats \
  -d "$GRAFT_REPO_ROOT/gpurun_out/prof_ug" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/scripts/time_env_ab.py" 27 1 > "$GRAFT_REPO_ROOT/gpurun_out/prof_ug.log" 2>&1 || exit 4
find "$GRAFT_REPO_ROOT/gpurun_out/prof_ug" -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} "$GRAFT_REPO_ROOT/gpurun_out/r4_kstats_ug.csv"
find "$GRAFT_REPO_ROOT/gpurun_out/prof_ug" -name "*kernel_trace.csv" -size +0 | head -1 | xargs -I{} cp {} "$GRAFT_REPO_ROOT/gpurun_out/r4_ktrace_ug.csv"
rm -rf "$GRAFT_REPO_ROOT/gpurun_out/prof_ug"
cd "$GRAFT_REPO_ROOT" || exit 9
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
for lib in ship pg2 pg6 pg8 pg12; do
  if [ "$lib" = ship ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$PWD/$V/libanomod_$lib.so; fi
  echo "== $lib"
  PPR_MODES=2 PPR_SUBS=1 timeout -k 10 120 python3 scripts/time_pagerank.py || exit 5
done > gpurun_out/r4_ppr_gather.log 2>&1
