#!/usr/bin/env python3
"""Edge-kernel stage time of the bench's span sets on whatever library
ANOMOD_LIB names (A/B of builds, run against run): SN 2^27 traces, the same
shuffled inside every trace, TrainTicket 2^27, LONG 2^23 (TS: the trace
structure of the SN set); per set the warm stage times and a digest of the
table.

  python scripts/experiments/r05/time_legs.py [reps] [sets, comma-separated]
"""
import hashlib
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[3]
sys.path[:0] = [str(ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"), str(ROOT)]

import anomod  # noqa: E402
from anomod import _lib as L  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
which = sys.argv[2].split(",") if len(sys.argv) > 2 else ["SN", "SNshuf", "TT", "LONG"]
lib = os.path.basename(os.environ.get("ANOMOD_LIB", "main"))
with anomod.Context(0) as ctx:
    for name in which:
        topo, lg = {"SN": ("SN", 27), "SNshuf": ("SN", 27), "TT": ("TT", 27), "LONG": ("LONG", 23),
                    "TS": ("SN", 27)}[name]
        dev = ctx.generate(anomod.SynthSpec(topo, seed=20251103, p_orphan_ppm=100), 1 << lg)
        if name == "SNshuf":
            d2 = ctx.shuffle(dev, seed=3)
            dev.free()
            dev = d2
        ms = []
        if name == "TS":  # trace structure of the SN set
            for r in range(reps + 1):
                ctx.trace_structure(dev, download=False)
                ms.append(ctx.stage_ms(L.STAGE_TRACE_STRUCT))
            print(json.dumps({"lib": lib, "set": name, "ms": [round(x, 3) for x in ms[1:]]}),
                  flush=True)
            dev.free()
            continue
        for r in range(reps + 1):
            t = ctx.edge_aggregate(dev, with_hist=True)
            ms.append(ctx.stage_ms(L.STAGE_EDGE_AGG))
        h = hashlib.sha256()
        for k in ("count", "errors", "sum_us", "min_us", "max_us", "hist"):
            h.update(getattr(t, k).tobytes())
        print(json.dumps({"lib": lib, "set": name, "ms": [round(x, 3) for x in ms[1:]],
                          "digest": h.hexdigest()[:16]}), flush=True)
        dev.free()
