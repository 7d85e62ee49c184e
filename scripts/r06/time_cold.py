#!/usr/bin/env python3
"""First-call anatomy of the ungrouped aggregation in the bench's order: the
headline set (2^27 SN traces) stays resident, an interleaved copy is made,
then three ungrouped aggregations; per call the wall, the stage events and
the host slots (anomod_ctx_host_ms) the call paid.  Then raw hipMalloc
timings of fresh device memory (first allocation vs a re-allocation).

  python scripts/r06/time_cold.py [traces_log2]
"""
import ctypes as C
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"), str(ROOT)]

import anomod  # noqa: E402
from anomod import _lib as L  # noqa: E402

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 27
out = {"traces": 1 << lg, "calls": []}
with anomod.Context(0) as ctx:
    t0 = time.perf_counter()
    spans = ctx.generate(anomod.SynthSpec("SN", seed=20251103, p_orphan_ppm=100), 1 << lg)
    ctx.synchronize()
    out["generate_ms"] = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    inter = ctx.shuffle(spans, seed=20251105, window_traces=4096)
    ctx.synchronize()
    out["shuffle_ms"] = (time.perf_counter() - t0) * 1e3
    for r in range(3):
        before = ctx.host_ms()
        t0 = time.perf_counter()
        ctx.edge_aggregate(inter, with_hist=False)
        wall = (time.perf_counter() - t0) * 1e3
        after = ctx.host_ms()
        paid = {k: round(v[0], 3) for k, v in after.items() if v[1] != before[k][1]}
        out["calls"].append({"wall_ms": round(wall, 3),
                             "group_ms": round(ctx.stage_ms(L.STAGE_GROUP), 3),
                             "edge_ms": round(ctx.stage_ms(L.STAGE_EDGE_AGG), 3), "host": paid})
        print(json.dumps(out["calls"][-1]), flush=True)
    inter.free()
    spans.free()

hip = C.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
hip.hipFree.argtypes = [C.c_void_p]
hip.hipDeviceSynchronize.argtypes = []
raw = []
for gb in (1, 8, 32, 8, 64):
    p = C.c_void_p()
    t0 = time.perf_counter()
    rc = hip.hipMalloc(C.byref(p), C.c_size_t(gb << 30))
    hip.hipDeviceSynchronize()
    ms = (time.perf_counter() - t0) * 1e3
    t1 = time.perf_counter()
    hip.hipFree(p)
    raw.append({"GiB": gb, "rc": rc, "malloc_ms": round(ms, 3),
                "free_ms": round((time.perf_counter() - t1) * 1e3, 3)})
    print(json.dumps(raw[-1]), flush=True)
out["raw_hipmalloc"] = raw
print(json.dumps(out))
