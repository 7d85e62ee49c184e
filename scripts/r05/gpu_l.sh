#!/bin/bash
# r05 call L: the upload pipeline tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5l
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_upload.py -m gpu -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/r5l/tests.log 2>&1 || exit 1
echo done
