#!/usr/bin/env python3
"""Time anomod_spans_group alone (2^lg SN traces interleaved in 4096-trace
windows) for the shipped library and every experiment build
csrc/build/variants/libanomod_gabl*.so (each in its own process)."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
PKG = ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"

if len(sys.argv) == 1 or sys.argv[1] != "--one":
    for lib in [None] + sorted(str(p) for p in (PKG / "csrc/build/variants").glob("libanomod_gabl*.so")):
        env = dict(os.environ)
        if lib:
            env["ANOMOD_LIB"] = lib
        r = subprocess.run([sys.executable, __file__, "--one"], env=env, timeout=300)
        if r.returncode:
            sys.exit(r.returncode)
    sys.exit(0)

sys.path[:0] = [str(PKG), str(ROOT)]
import numpy as np  # noqa: E402

import anomod  # noqa: E402
from anomod import _lib as L  # noqa: E402

lg = int(os.environ.get("GRP_LG", 25))
with anomod.Context(0) as ctx:
    dev = ctx.generate(anomod.SynthSpec("SN", seed=20251103, p_orphan_ppm=100), 1 << lg)
    inter = ctx.shuffle(dev, seed=5, window_traces=4096)
    n = dev.n_spans
    dev.free()
    ms = []
    for _ in range(4):
        g = ctx.group(inter)
        ms.append(ctx.stage_ms(L.STAGE_GROUP))
        g.free()
    print(json.dumps({"lib": os.environ.get("ANOMOD_LIB", "main").split("/")[-1], "spans": n,
                      "group_ms": ms[1:], "gspans_per_s": n / np.median(ms[1:]) / 1e6}), flush=True)
