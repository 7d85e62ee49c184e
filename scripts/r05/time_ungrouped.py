#!/usr/bin/env python3
"""The bench's ungrouped leg on whatever library ANOMOD_LIB names: 2^27 SN
traces with the spans of every 4096 consecutive traces interleaved; per call
the grouping and table stage times, and a digest of the table.

  python scripts/r05/time_ungrouped.py [reps]
"""
import hashlib
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"), str(ROOT)]

import anomod  # noqa: E402
from anomod import _lib as L  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
with anomod.Context(0) as ctx:
    dev = ctx.generate(anomod.SynthSpec("SN", seed=20251103, p_orphan_ppm=100), 1 << 27)
    inter = ctx.shuffle(dev, seed=20251105, window_traces=4096)
    dev.free()
    g, e = [], []
    for r in range(reps + 1):
        t = ctx.edge_aggregate(inter, with_hist=True)
        g.append(ctx.stage_ms(L.STAGE_GROUP))
        e.append(ctx.stage_ms(L.STAGE_EDGE_AGG))
    h = hashlib.sha256()
    for k in ("count", "errors", "sum_us", "min_us", "max_us", "hist"):
        h.update(getattr(t, k).tobytes())
    print(json.dumps({"lib": os.path.basename(os.environ.get("ANOMOD_LIB", "main")),
                      "group_ms": [round(x, 3) for x in g[1:]], "edge_ms": [round(x, 3) for x in e[1:]],
                      "digest": h.hexdigest()[:16]}), flush=True)
