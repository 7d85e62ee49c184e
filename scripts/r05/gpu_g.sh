#!/bin/bash
# r05 call G: the whole GPU suite, then the profile of the bench process
# (kernel trace + stats) and the PMC passes (scripts/profile_r05.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5g
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r5g/gpu_tests.log 2>&1 || exit 1
bash scripts/profile_r05.sh $GRAFT_REPO_ROOT/gpurun_out/r05prof || exit 2
echo done
