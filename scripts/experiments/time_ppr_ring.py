#!/usr/bin/env python3
"""Persistent PageRank solve with the per-iteration vector ring (default) vs
the two-buffer form (ANOMOD_PPR_RING=0), alternating in one process on the
bench's config-5 graph; every vector compared bit for bit with the per-launch
path (ANOMOD_PPR_MODE=1)."""
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

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
with anomod.Context(0) as ctx:
    for n_nodes in (100_000, 20_000):
        g = anomod.DeviceGraph(ctx, synthetic=(n_nodes, 10, 11))
        rng = np.random.default_rng(n_nodes)
        for iters, tol in ((100, 0.0), (1000, 1e-10)):
            ps = [rng.random(g.N) for _ in range(reps)]
            os.environ["ANOMOD_PPR_MODE"] = "1"
            refs = [g.pagerank(p, iters=iters, tol=tol) for p in ps]
            os.environ["ANOMOD_PPR_MODE"] = "2"
            res = {}
            for r in range(reps):
                for ring in ("1", "0"):
                    os.environ["ANOMOD_PPR_RING"] = ring
                    t = time.perf_counter()
                    x, it = g.pagerank(ps[r], iters=iters, tol=tol)
                    wall = (time.perf_counter() - t) * 1e3
                    ok = bool(np.array_equal(x, refs[r][0]) and it == refs[r][1])
                    k = ctx.stage_ms(L.STAGE_PAGERANK)
                    res.setdefault(ring, []).append([round(k * 1e3 / it, 3), round(wall, 3), ok,
                                                     g.last_solve()[0]])
            print(json.dumps({"N": g.N, "iters": iters, "tol": tol,
                              "ring_us_per_iter_wall_equal_path": res["1"],
                              "two_buffer": res["0"]}), flush=True)
        g.free()
