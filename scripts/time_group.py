#!/usr/bin/env python3
"""Time the ungrouped path (trace grouping + edge aggregation) and the
grouped edge kernel on in-trace-shuffled / TrainTicket sets.

  python scripts/time_group.py [log2_traces] [reps]
"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"), str(ROOT)]

import numpy as np  # noqa: E402

import anomod  # noqa: E402
from anomod import _lib as L  # noqa: E402

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 25
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
out = {}
with anomod.Context(0) as ctx:
    for topo in ("SN", "TT"):
        dev = ctx.generate(anomod.SynthSpec(topo, seed=20251103, p_orphan_ppm=100), 1 << lg)
        n, nt = dev.n_spans, dev.n_traces
        ctx.edge_aggregate(dev, with_hist=False)
        ms = []
        for _ in range(reps):
            ctx.edge_aggregate(dev, with_hist=False)
            ms.append(ctx.stage_ms(L.STAGE_EDGE_AGG))
        rec = {"spans": n, "traces": nt, "grouped_edge_ms": ms}
        intra = ctx.shuffle(dev, seed=3, window_traces=0)
        ctx.edge_aggregate(intra, with_hist=False)
        ms = []
        for _ in range(reps):
            ctx.edge_aggregate(intra, with_hist=False)
            ms.append(ctx.stage_ms(L.STAGE_EDGE_AGG))
        rec["intra_shuffled_edge_ms"] = ms
        intra.free()
        if topo == "SN":
            inter = ctx.shuffle(dev, seed=5, window_traces=4096)
            dev.free()
            ctx.edge_aggregate(inter, with_hist=False)
            g, e, wall = [], [], []
            for _ in range(reps):
                t0 = time.perf_counter()
                ctx.edge_aggregate(inter, with_hist=False)
                wall.append((time.perf_counter() - t0) * 1e3)
                g.append(ctx.stage_ms(L.STAGE_GROUP))
                e.append(ctx.stage_ms(L.STAGE_EDGE_AGG))
            rec.update(group_ms=g, ungrouped_edge_ms=e, ungrouped_wall_ms=wall)
            inter.free()
        else:
            dev.free()
        out[topo] = rec
        print(json.dumps({topo: rec}), flush=True)
