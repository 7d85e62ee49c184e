#!/bin/bash
# r05 call S: aliased-id chunk tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5s
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_edge.py -m gpu -x -v --timeout 120 \
  --timeout-method thread -k "alias or fingerprint" > gpurun_out/r5s/tests.log 2>&1 || exit 1
echo done
