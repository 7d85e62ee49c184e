#!/bin/bash
# r04 final profile: bench process under rocprofv3 (trace + stats), PMC passes,
# each step time-limited (scripts/profile_r04.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
bash scripts/profile_r04.sh "$GRAFT_REPO_ROOT/gpurun_out/r04prof" > gpurun_out/r04prof.log 2>&1
