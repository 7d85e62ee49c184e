#!/usr/bin/env python3
"""Time PageRank solves on the bench's config-5 graph (N = 1e5, ~7e5 edges):
auto / per-iteration launches (ANOMOD_PPR_MODE=1) / persistent one-launch solve (2), the
persistent one with 1, 2 or 4 256-row blocks per workgroup (ANOMOD_PPR_SUB, PPR_SUBS)."""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"), str(ROOT)]
import numpy as np  # noqa: E402

import anomod  # noqa: E402
from anomod import _lib as L  # noqa: E402

with anomod.Context(0) as ctx:
  for n_nodes in [int(v) for v in os.environ.get("PPR_NS", "100000").split(",")]:
    g = anomod.DeviceGraph(ctx, synthetic=(n_nodes, 10, 11))
    p = np.random.default_rng(0).random(g.N)
    ref = {}
    for mode, sub in [(m, s) for m in os.environ.get("PPR_MODES", "0,1,2").split(",")
                      for s in (os.environ.get("PPR_SUBS", "1,2,4").split(",") if m == "2" else ["default"])]:
        os.environ["ANOMOD_PPR_MODE"] = mode
        if sub == "default":
            os.environ.pop("ANOMOD_PPR_SUB", None)
        else:
            os.environ["ANOMOD_PPR_SUB"] = sub
        for iters, tol in ((100, 0.0), (1000, 1e-10)):
            x, _ = g.pagerank(p, iters=iters, tol=tol)
            same = bool(np.array_equal(ref.setdefault((iters, tol), x), x))
            ms, wall, its = [], [], 0
            for _ in range(5):
                t = time.perf_counter()
                _, its = g.pagerank(p, iters=iters, tol=tol)
                wall.append((time.perf_counter() - t) * 1e3)
                ms.append(ctx.stage_ms(L.STAGE_PAGERANK))
            k = float(np.median(ms))
            print(json.dumps({"N": g.N, "mode": mode, "sub": sub, "bits_equal": same,
                              "iters": its, "tol": tol, "kernel_ms": k,
                              "us_per_iter": k * 1e3 / its, "iters_per_s": its / k * 1e3,
                              "wall_ms": float(np.median(wall))}), flush=True)
    g.free()
