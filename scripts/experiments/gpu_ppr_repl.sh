#!/bin/bash
# PageRank grid barrier: copies of the top counter (shipped 8; r0 = one line
# polled by every block, r16/r32/r64) and the spin's sleep (s0 = none), N = 1e5
# / 2e4 with the ring, every vector compared with the per-launch path.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
for lib in ${LIBS:-ship r0 r16 r32 r64 s0 r32s0 ship}; do
  if [ "$lib" = ship ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$PWD/$V/libanomod_$lib.so; fi
  echo "== $lib"
  timeout -k 10 120 python3 scripts/experiments/time_ppr_ring.py 5 || exit 1
  [ -n "$BATCH" ] && { timeout -k 10 120 python3 scripts/experiments/time_ppr_batch.py || exit 1; }
done
exit 0
