#!/usr/bin/env python3
"""Sequential EWMA kernel at the config-4 chunk shape (S = 10^5, T = 131 040,
W = 60) for several ANOMOD_EWMA_SEG launch segments, each in its own process."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
if len(sys.argv) == 1:
    for seg in os.environ.get("SEGS", "0 16384 32768 65536 8192").split():
        env = dict(os.environ, ANOMOD_EWMA_SEG=seg, ANOMOD_EWMA_MODE="1")
        for _ in range(int(os.environ.get("REPS", 2))):
            r = subprocess.run([sys.executable, __file__, "--one"], env=env, timeout=300)
            if r.returncode:
                sys.exit(r.returncode)
    sys.exit(0)

sys.path[:0] = [str(ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"), str(ROOT)]
import numpy as np  # noqa: E402

import anomod  # noqa: E402
from anomod import _lib as L  # noqa: E402

S, T, W = 100000, 131040, 60
with anomod.Context(0) as ctx:
    ser = anomod.DeviceSeries(ctx, T, S)
    ser.fill_synthetic(7, 0)
    ser.ewma_z(2 / (W + 1), W, download=False)
    ms = []
    for c in range(4):
        ser.fill_synthetic(7, c * T)
        ser.ewma_z(2 / (W + 1), W, download=False)
        ms.append(ctx.stage_ms(L.STAGE_EWMA))
    k = float(np.median(ms))
    print(json.dumps({"seg": os.environ["ANOMOD_EWMA_SEG"], "kernel_ms": round(k, 3),
                      "all": [round(x, 2) for x in ms],
                      "GBps": round((4 * T * S + 4 * (T // W) * S + 40 * S) / k / 1e6)}), flush=True)
    ser.free()
