#!/usr/bin/env python3
"""Time the sequential EWMA/z kernel (ANOMOD_EWMA_MODE=1, tiled layout) at the
bench's config-4 chunk shape (S = 10^5, T = 131 040, W = 60) and at T = 7680,
for the shipped library and every experiment build
csrc/build/variants/libanomod_ew*.so (each in its own process)."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
PKG = ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"

if len(sys.argv) == 1 or sys.argv[1] != "--one":
    for lib in [None] + sorted(str(p) for p in (PKG / "csrc/build/variants").glob("libanomod_ew*.so")):
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

os.environ["ANOMOD_EWMA_MODE"] = "1"
S, W = 100000, 60
with anomod.Context(0) as ctx:
    for T in (131040, 7680):
        ser = anomod.DeviceSeries(ctx, T, S)
        ser.fill_synthetic(7, 0)
        ser.ewma_z(2 / (W + 1), W, download=False)
        ms = []
        for c in range(4):
            ser.fill_synthetic(7, c * T)
            ser.ewma_z(2 / (W + 1), W, download=False)
            ms.append(ctx.stage_ms(L.STAGE_EWMA))
        k = float(np.median(ms))
        b = 4 * T * S + 4 * (T // W) * S + 40 * S
        print(json.dumps({"lib": os.environ.get("ANOMOD_LIB", "main").split("/")[-1], "T": T,
                          "kernel_ms": k, "GBps": b / k / 1e6}), flush=True)
        ser.free()
