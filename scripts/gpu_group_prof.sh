#!/bin/bash
# Kernel-time breakdown of the grouping paths (rocprofv3 --kernel-trace --stats).
cd "$GRAFT_REPO_ROOT" || exit 9
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-g}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$T" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/scripts/time_group_paths.py" ${LG:-25} 2 ${AVGS:-1024} > "$GRAFT_REPO_ROOT/gpurun_out/prof_$T.log" 2>&1 || exit $?
find "$GRAFT_REPO_ROOT/gpurun_out/prof_$T" -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} "$GRAFT_REPO_ROOT/gpurun_out/kstats_$T.csv"
find "$GRAFT_REPO_ROOT/gpurun_out/prof_$T" -name "*kernel_trace.csv" -size +0 | head -1 | xargs -I{} cp {} "$GRAFT_REPO_ROOT/gpurun_out/ktrace_$T.csv"
rm -rf "$GRAFT_REPO_ROOT/gpurun_out/prof_$T"
