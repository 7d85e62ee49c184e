#!/bin/bash
# Bucket-path A/B: kernel traces of the shipped build and the experiment-only
# builds of bucket.hip (csrc/build/variants/libanomod_<v>.so) on the same set.
cd "$GRAFT_REPO_ROOT" || exit 9
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp TG_NO_LSD=1
cd /tmp
for v in ship ${VARS:-bk1 bk2 bk4 bk5}; do
  if [ "$v" = ship ]; then unset ANOMOD_LIB; else
    export ANOMOD_LIB="$R/anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants/libanomod_$v.so"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/ab_$v" -o run --output-format csv -- \
    python3 "$R/scripts/experiments/time_group_paths.py" ${LG:-25} 2 ${AVGS:-1400} > "$R/gpurun_out/ab_$v.log" 2>&1 || exit $?
  f=$(find "$R/gpurun_out/ab_$v" -name "*kernel_trace.csv" | head -1)
  python3 "$R/scripts/ktrace_summary.py" "$f" bk_ > "$R/gpurun_out/ab_$v.txt"
  rm -rf "$R/gpurun_out/ab_$v"
done
