#!/bin/bash
# Stage times of the native metric-CSV decoder (host only): builds a harness
# around csrc/metrics_decode.cpp with -DANOMOD_DECODE_TIMING (stage marks to
# stderr; the library build has none) and runs it on one staged config-2
# experiment CSV at the given thread counts.
#   bash scripts/r06/decode_stages.sh OUTDIR [threads ...]
set -e
cd "$(dirname "$0")/../.."
out=${1:-/tmp}; shift || true
g++ -O3 -march=x86-64-v2 -std=c++17 -DANOMOD_DECODE_TIMING -o "$out/decode_stages" \
  scripts/r06/decode_stages_main.cpp \
  anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/metrics_decode.cpp -lpthread
csv=$(python3 -c "
import sys, tempfile
sys.path[:0] = ['anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd', '.']
import bench
print(bench._stage_tt_experiment((tempfile.mkdtemp(prefix='anomod_dec_'), 0, bench.TT_FAULTS[0]))[1])")
for t in "${@:-16}"; do
  echo "threads $t"
  ANOMOD_DECODE_THREADS=$t "$out/decode_stages" "$csv" 2>&1
done
