#!/bin/bash
# r05 call J: smoke, then the plain default bench (the driver's command).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r5j
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > gpurun_out/r5j/smoke.log 2>&1 || exit 1
timeout -k 10 900 python3 -u bench.py > gpurun_out/r5j/bench.log 2> gpurun_out/r5j/bench.err || exit 2
echo done
