#!/usr/bin/env python3
"""Grouping time of the bucket path vs the LSD path on the same interleaved
SN set (spans of every 4096 consecutive traces interleaved), alternating.

  python scripts/experiments/time_group_paths.py [log2_traces] [reps] [avg ...]
"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"), str(ROOT)]

import anomod  # noqa: E402
from anomod import _lib as L  # noqa: E402

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 25
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
avgs = sys.argv[3:] or ["1024"]
with anomod.Context(0) as ctx:
    topo = os.environ.get("TG_TOPO", "SN")
    dev = ctx.generate(anomod.SynthSpec(topo, seed=20251103, p_orphan_ppm=100), 1 << lg)
    want = ctx.edge_aggregate(dev, with_hist=False)
    inter = ctx.shuffle(dev, seed=5, window_traces=4096)
    n = dev.n_spans
    dev.free()
    res = {"spans": n, "traces": 1 << lg}
    variants = ([] if os.environ.get("TG_NO_LSD") else [("lsd", None)]) + \
        [("bucket", a) for a in avgs]
    for r in range(reps):
        for path, avg in variants:
            os.environ["ANOMOD_GROUP_PATH"] = path
            if avg:
                os.environ["ANOMOD_BUCKET_AVG"] = avg
            t = ctx.edge_aggregate(inter, with_hist=False)
            key = path if avg is None else f"bucket_{avg}"
            res.setdefault(key + "_group_ms", []).append(round(ctx.stage_ms(L.STAGE_GROUP), 3))
            res.setdefault(key + "_edge_ms", []).append(round(ctx.stage_ms(L.STAGE_EDGE_AGG), 3))
            ok = all((getattr(t, k) == getattr(want, k)).all()
                     for k in ("count", "errors", "sum_us", "min_us", "max_us"))
            res.setdefault(key + "_equal", []).append(bool(ok))
            res[key + "_info"] = ctx.group_info()
            print(json.dumps({key: res[key + "_group_ms"][-1], "equal": ok}), flush=True)
    print(json.dumps(res), flush=True)
