#!/bin/bash
# Join-kernel variants (build/variants/libanomod_<name>.so) against the
# shipped library: the fused ungrouped aggregation at 2^27 SN traces, each in
# its own process, alternating; then the fused tests under each variant.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
for lib in ${LIBS:-ship jp3 ship jp3}; do
  if [ "$lib" = ship ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$PWD/$V/libanomod_$lib.so; fi
  echo "== $lib"
  AB_VAR=ANOMOD_UNGROUPED_FUSED AB_VALS=1 timeout -k 10 200 python3 scripts/time_env_ab.py 27 3 | tail -1 || exit 1
done
for lib in ${LIBS:-jp3}; do
  [ "$lib" = ship ] && continue
  export ANOMOD_LIB=$PWD/$V/libanomod_$lib.so
  timeout -k 10 200 python3 -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_group.py | tail -1 || exit 2
done
exit 0
