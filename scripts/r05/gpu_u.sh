#!/bin/bash
# r05 call U: the whole GPU suite on the final tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5u
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r5u/gpu_tests.log 2>&1 || exit 1
echo done
