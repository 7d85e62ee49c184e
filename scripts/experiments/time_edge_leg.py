#!/usr/bin/env python3
"""Edge-aggregation kernel time of one synthetic leg (TG_TOPO = SN / TT /
LONG, 2^lg traces) under the library ANOMOD_LIB points at: warm-up, then
`reps` timed calls; prints ms per call and a digest of the table, so builds
can be compared for time and bits.

  ANOMOD_LIB=... TG_TOPO=LONG python scripts/experiments/time_edge_leg.py 23 5
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

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 23
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
topo = os.environ.get("TG_TOPO", "LONG")
with anomod.Context(0) as ctx:
    dev = ctx.generate(anomod.SynthSpec(topo, seed=20251103, p_orphan_ppm=100), 1 << lg)
    t = ctx.edge_aggregate(dev, with_hist=True)
    first = ctx.stage_ms(L.STAGE_EDGE_AGG)
    ms = []
    for _ in range(reps):
        t = ctx.edge_aggregate(dev, with_hist=True)
        ms.append(round(ctx.stage_ms(L.STAGE_EDGE_AGG), 3))
    h = hashlib.sha256()
    for k in ("count", "errors", "sum_us", "min_us", "max_us", "hist"):
        h.update(getattr(t, k).tobytes())
    print(json.dumps({"lib": Path(os.environ.get("ANOMOD_LIB", "libanomod.so")).name, "topo": topo,
                      "spans": dev.n_spans, "first_ms": round(first, 3), "ms": ms,
                      "digest": h.hexdigest()[:16]}), flush=True)
