#!/usr/bin/env python3
"""Probe: one tolerance-mode PageRank (cooperative persistent launch) and exit;
run under rocprofv3 --kernel-trace to see whether the profiler's teardown
survives a process that made a cooperative launch."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"), str(ROOT)]
import numpy as np  # noqa: E402

import anomod  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "coop"
with anomod.Context(0) as ctx:
    g = anomod.DeviceGraph(ctx, synthetic=(20000, 8, 1))
    p = np.random.default_rng(0).random(g.N)
    x, it = g.pagerank(p, iters=1000, tol=1e-10 if mode == "coop" else 0.0)
    g.free()
print("probe", mode, it, flush=True)
