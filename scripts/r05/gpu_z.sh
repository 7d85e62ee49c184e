#!/bin/bash
# r05 call Z (final library): the whole GPU suite, smoke, the plain default
# bench, then the profile of the bench process and the PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5z
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r5z/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > gpurun_out/r5z/smoke.log 2>&1 || exit 2
timeout -k 10 900 python3 -u bench.py > gpurun_out/r5z/bench.log 2> gpurun_out/r5z/bench.err || exit 3
bash scripts/profile_r05.sh $GRAFT_REPO_ROOT/gpurun_out/r05prof || exit 4
echo done
