#!/usr/bin/env python3
"""Probe: does the sequential EWMA kernel's time depend on which allocation
holds X?  Several DeviceSeries of the same shape in one process, each timed
twice, interleaved (S = 10^5, T = 32 760, W = 60, mode 1)."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"), str(ROOT)]
import numpy as np  # noqa: E402

import anomod  # noqa: E402
from anomod import _lib as L  # noqa: E402

os.environ["ANOMOD_EWMA_MODE"] = "1"
S, T, W = 100000, 32760, 60
with anomod.Context(0) as ctx:
    sers = [anomod.DeviceSeries(ctx, T, S) for _ in range(4)]
    for k, s in enumerate(sers):
        s.fill_synthetic(7, 0)
        s.ewma_z(2 / (W + 1), W, download=False)
    for rnd in range(3):
        for k, s in enumerate(sers):
            s.reset_state()
            s.ewma_z(2 / (W + 1), W, download=False)
            ms = ctx.stage_ms(L.STAGE_EWMA)
            print(json.dumps({"round": rnd, "alloc": k, "ms": round(ms, 3),
                              "GBps": round(4 * T * S / ms / 1e6)}), flush=True)
    for s in sers:
        s.free()
