#!/bin/bash
# Kernel trace of one command: bash scripts/gpu_ktrace.sh TAG FILTER -- cmd...
# -> gpurun_out/kt_TAG.txt (per-dispatch name / grid / ms, scripts/ktrace_summary.py)
R="$GRAFT_REPO_ROOT"
T=$1; F=$2; shift 3
rm -rf "$R/gpurun_out/kt_$T" "$R/gpurun_out/kt_$T.txt"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/kt_$T" -o run --output-format csv -- "$@" > "$R/gpurun_out/kt_$T.log" 2>&1 || exit $?
f=$(find "$R/gpurun_out/kt_$T" -name "*kernel_trace.csv" | head -1)
python3 "$R/scripts/ktrace_summary.py" "$f" "$F" > "$R/gpurun_out/kt_$T.txt"
rm -rf "$R/gpurun_out/kt_$T"
