#!/usr/bin/env python3
"""Time the trace-structure kernel on synthetic SN spans resident in HBM
(the bench's extras leg at a configurable size); with no argument, also every
experiment-only build csrc/build/variants/libanomod_ts*.so, each in its own
process (ANOMOD_LIB)."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"), str(ROOT)]
import numpy as np  # noqa: E402

import anomod  # noqa: E402
from anomod import _lib as L  # noqa: E402

if len(sys.argv) == 1:
    pkg = ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"
    for lib in [None] + sorted(str(p) for p in (pkg / "csrc/build/variants").glob("libanomod_ts*.so")):
        env = dict(os.environ)
        if lib:
            env["ANOMOD_LIB"] = lib
        r = subprocess.run([sys.executable, __file__, "--one"], env=env, timeout=200)
        if r.returncode:
            sys.exit(r.returncode)
    sys.exit(0)

traces = int(os.environ.get("TS_TRACES", 1 << 25))
with anomod.Context(0) as ctx:
    sp = ctx.generate(anomod.SynthSpec("SN", seed=20251103, p_orphan_ppm=100), traces)
    ctx.trace_structure(sp, download=False)
    ms = []
    for _ in range(5):
        ctx.trace_structure(sp, download=False)
        ms.append(ctx.stage_ms(L.STAGE_TRACE_STRUCT))
    k = float(np.median(ms))
    b = 33 * sp.n_spans + 20 * sp.n_traces
    print(json.dumps({"lib": os.environ.get("ANOMOD_LIB", "main"), "spans": sp.n_spans,
                      "kernel_ms": k, "gspans_per_s": sp.n_spans / k / 1e6,
                      "GBps": b / k / 1e6}), flush=True)
