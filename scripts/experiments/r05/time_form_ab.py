#!/usr/bin/env python3
"""First-call cost of the headline set: the edge kernel's auto form (pair
table with the saturation hand-off, what a set's first aggregation runs)
against the plain pair form, alternating in one process on a warm set, plus
the cold first call itself:

  python scripts/experiments/r05/time_form_ab.py [log2_traces] [reps] [topo] [shuffle]
"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[3]
sys.path[:0] = [str(ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"), str(ROOT)]

import anomod  # noqa: E402
from anomod import _lib as L  # noqa: E402

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 27
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
topo = sys.argv[3] if len(sys.argv) > 3 else "SN"
shuffle = len(sys.argv) > 4 and sys.argv[4] == "1"
touch = len(sys.argv) > 5 and sys.argv[5] == "1"  # read the set once (trace structure) first
with anomod.Context(0) as ctx:
    dev = ctx.generate(anomod.SynthSpec(topo, seed=20251103, p_orphan_ppm=100), 1 << lg)
    if shuffle:
        d2 = ctx.shuffle(dev, seed=3)
        dev.free()
        dev = d2
    if touch:
        ctx.trace_structure(dev, download=False)
    t = ctx.edge_aggregate(dev, with_hist=False)
    print(json.dumps({"touched": touch, "cold_ms": round(ctx.stage_ms(L.STAGE_EDGE_AGG), 3), "hints": dev.hints}),
          flush=True)
    for r in range(reps):
        for form in ("auto", "pair", "default"):
            if form == "default":
                os.environ.pop("ANOMOD_HIST_FORM", None)
            else:
                os.environ["ANOMOD_HIST_FORM"] = form
            t2 = ctx.edge_aggregate(dev, with_hist=False)
            ok = all((getattr(t, k) == getattr(t2, k)).all() for k in ("count", "sum_us"))
            print(json.dumps({"form": form, "ms": round(ctx.stage_ms(L.STAGE_EDGE_AGG), 3),
                              "equal": bool(ok)}), flush=True)
