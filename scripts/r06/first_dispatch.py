#!/usr/bin/env python3
"""First vs later aggregations of a freshly generated set (the bench's TT and
LONG legs): per call the edge stage time and wall.  Run under
`rocprofv3 --kernel-trace` to see every dispatch of the same instantiation.

  python scripts/r06/first_dispatch.py [TT|LONG|SN] [traces_log2] [calls]
"""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"), str(ROOT)]

import anomod  # noqa: E402
from anomod import _lib as L  # noqa: E402

topo = sys.argv[1] if len(sys.argv) > 1 else "TT"
lg = int(sys.argv[2]) if len(sys.argv) > 2 else (27 if topo != "LONG" else 23)
calls = int(sys.argv[3]) if len(sys.argv) > 3 else 4
with anomod.Context(0) as ctx:
    if os.environ.get("PRE_SN"):  # the bench's order: the headline set came and went first
        s0 = ctx.generate(anomod.SynthSpec("SN", seed=20251103, p_orphan_ppm=100), 1 << 27)
        ctx.edge_aggregate(s0, with_hist=False)
        s0.free()
    t0 = time.perf_counter()
    s = ctx.generate(anomod.SynthSpec(topo, seed=20251103, p_orphan_ppm=100), 1 << lg)
    ctx.synchronize()
    gen = (time.perf_counter() - t0) * 1e3
    res = []
    for r in range(calls):
        t0 = time.perf_counter()
        ctx.edge_aggregate(s, with_hist=False)
        res.append({"wall_ms": round((time.perf_counter() - t0) * 1e3, 3),
                    "kernel_ms": round(ctx.stage_ms(L.STAGE_EDGE_AGG), 3)})
    print(json.dumps({"topo": topo, "traces": 1 << lg, "spans": s.n_spans, "generate_ms": gen,
                      "calls": res}), flush=True)
    s.free()
