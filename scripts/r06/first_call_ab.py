#!/usr/bin/env python3
"""What a freshly generated set's first aggregation pays:
per topology, the edge stage of four calls right after generation, after the
GPU idled 2 s, and after 40 GB of device-to-device copies (memory clocks busy);
then the warm time of each histogram form forced (pair / compact).

  python scripts/r06/first_call_ab.py [TT|SN|LONG] [log2_traces]
"""
import ctypes as C
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
lg = int(sys.argv[2]) if len(sys.argv) > 2 else (23 if topo == "LONG" else 27)
hip = C.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]


def calls(ctx, s, k=4):
    out = []
    for _ in range(k):
        ctx.edge_aggregate(s, with_hist=False)
        out.append(round(ctx.stage_ms(L.STAGE_EDGE_AGG), 3))
    return out


with anomod.Context(0) as ctx:
    spec = anomod.SynthSpec(topo, seed=20251103, p_orphan_ppm=100)
    a, b = C.c_void_p(), C.c_void_p()
    assert hip.hipMalloc(C.byref(a), 8 << 30) == 0 and hip.hipMalloc(C.byref(b), 8 << 30) == 0
    res = {"topo": topo, "traces": 1 << lg}
    for mode in ("right_after", "idle_2s", "after_copies", "right_after_again"):
        s = ctx.generate(spec, 1 << lg)
        ctx.synchronize()
        if mode == "idle_2s":
            time.sleep(2.0)
        elif mode == "after_copies":
            for _ in range(5):
                hip.hipMemcpy(b, a, 8 << 30, 3)
        res[mode] = calls(ctx, s)
        res[mode + "_hints"] = s.hints
        print(json.dumps({mode: res[mode], "hints": s.hints}), flush=True)
        if mode != "right_after_again":
            s.free()
    for form in ("pair", "compact"):
        os.environ["ANOMOD_HIST_FORM"] = form
        res["warm_" + form] = calls(ctx, s, 3)
        print(json.dumps({form: res["warm_" + form]}), flush=True)
    del os.environ["ANOMOD_HIST_FORM"]
    s.free()
    print(json.dumps(res), flush=True)
