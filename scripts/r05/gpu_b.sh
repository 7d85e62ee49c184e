#!/bin/bash
# r05 call B: the whole GPU suite; join occupancy A/B (same process); the
# first-call (auto hist form) A/B on SN; host-set upload timing (LONG 2^20
# traces); PageRank batch K = 8 / 16; the counters rocprofv3 offers.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 9
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || exit 1
AB_VAR=ANOMOD_JOIN_W6 AB_VALS=0,1,2 timeout -k 10 240 python3 -u scripts/time_env_ab.py 27 3 \
  > $O/ab_w6.log 2>&1 || exit 2
timeout -k 10 240 python3 -u scripts/r05/time_form_ab.py 27 3 SN > $O/form_sn.log 2>&1 || exit 3
timeout -k 10 240 python3 -u scripts/r05/time_form_ab.py 27 3 SN 1 > $O/form_sn_shuf.log 2>&1 || exit 4
timeout -k 10 300 python3 -u bench.py --legs long_traces,pagerank,ungrouped --steps 3 --warmup 1 --no-cpu-baseline --leg-cpu-seconds 3 > $O/bench_lp.log 2>&1 || exit 5
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
echo done
