#!/bin/bash
# r04 final: the whole GPU suite, the default bench (plain), then the profile
# (bench under rocprofv3 + PMC passes) of the same tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r4final_t.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py > gpurun_out/r4final_bench.json 2> gpurun_out/r4final_bench.err || exit 2
bash scripts/profile_r04.sh "$GRAFT_REPO_ROOT/gpurun_out/r04final" > gpurun_out/r04final.log 2>&1 || exit 3
