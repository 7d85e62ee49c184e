#!/usr/bin/env python3
"""The LONG leg (bench.py long_traces: 2^23 traces) on whatever library
ANOMOD_LIB names: per-call stage time and a digest of the table, so builds
can be compared run against run:

  python scripts/experiments/r05/time_long.py [log2_traces] [reps]
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

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 23
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
with anomod.Context(0) as ctx:
    dev = ctx.generate(anomod.SynthSpec("LONG", seed=20251103, p_orphan_ppm=100), 1 << lg)
    ms = []
    for r in range(reps + 1):
        t = ctx.edge_aggregate(dev, with_hist=True)
        ms.append(ctx.stage_ms(L.STAGE_EDGE_AGG))
    h = hashlib.sha256()
    for k in ("count", "errors", "sum_us", "min_us", "max_us", "hist"):
        h.update(getattr(t, k).tobytes())
    print(json.dumps({"lib": os.path.basename(os.environ.get("ANOMOD_LIB", "main")),
                      "cold_ms": round(ms[0], 3), "ms": [round(x, 3) for x in ms[1:]],
                      "digest": h.hexdigest()[:16]}), flush=True)
