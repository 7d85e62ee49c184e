#!/bin/bash
# r05 call N: the select-built parent scan per table form and the scan
# widths around it (TT: kFwd / kBwd; LONG: kLFwd / kLBwd), trace structure
# with it; two alternating rounds, digests compared across builds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5n
V=anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd/csrc/build/variants
: > gpurun_out/r5n/legs.log
run() {  # lib sets
  if [ $1 = main ]; then unset ANOMOD_LIB; else export ANOMOD_LIB=$GRAFT_REPO_ROOT/$V/libanomod_$1.so; fi
  timeout -k 10 200 python3 -u scripts/r05/time_legs.py 4 $2 >> gpurun_out/r5n/legs.log 2>&1
}
for round in 1 2; do
  run main SN,SNshuf,TT,LONG,TS || exit 1
  run old SN,TT,LONG || exit 1
  run selsn SN,SNshuf || exit 1
  for v in tt84 tt66 tt44; do run $v TT || exit 1; done
  for v in l106 l66 l124; do run $v LONG || exit 1; done
  run ts1 TS || exit 1
done
echo done
