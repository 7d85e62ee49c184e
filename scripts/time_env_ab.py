#!/usr/bin/env python3
"""Grouping + edge time of the ungrouped SN set (spans of every 4096
consecutive traces interleaved) under alternating values of one run-time
knob, same process, same set:

  AB_VAR=ANOMOD_BK_XCD AB_VALS=0,3 python scripts/time_env_ab.py [log2_traces] [reps]
"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"), str(ROOT)]

import anomod  # noqa: E402
from anomod import _lib as L  # noqa: E402

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 25
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
var = os.environ.get("AB_VAR", "ANOMOD_BK_XCD")
vals = os.environ.get("AB_VALS", "0,3").split(",")
with anomod.Context(0) as ctx:
    dev = ctx.generate(anomod.SynthSpec(os.environ.get("TG_TOPO", "SN"), seed=20251103,
                                        p_orphan_ppm=100), 1 << lg)
    want = ctx.edge_aggregate(dev, with_hist=False)
    inter = ctx.shuffle(dev, seed=5, window_traces=4096)
    dev.free()
    res = {"var": var, "traces": 1 << lg}
    for r in range(reps):
        for v in vals:
            os.environ[var] = v
            t = ctx.edge_aggregate(inter, with_hist=False)
            ok = all((getattr(t, k) == getattr(want, k)).all()
                     for k in ("count", "errors", "sum_us", "min_us", "max_us"))
            g, e = round(ctx.stage_ms(L.STAGE_GROUP), 3), round(ctx.stage_ms(L.STAGE_EDGE_AGG), 3)
            res.setdefault(v, []).append([g, e, ok])
            print(json.dumps({var: v, "group_ms": g, "edge_ms": e, "equal": ok}), flush=True)
    print(json.dumps(res), flush=True)
