#!/usr/bin/env python3
"""The two native decoders of one config-2 experiment, timed apart (host
only, no GPU): the SkyWalking collector payload (JSON, indent=2, ~20 MB) and
the long metric CSV (~215 MB), each file decoded 5 times from the page cache.

  python scripts/r06/time_decode.py [threads,...]"""
import json
import os
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"), str(ROOT)]

import bench  # noqa: E402
from anomod import decode  # noqa: E402

threads = sys.argv[1].split(",") if len(sys.argv) > 1 else ["1", "8", "16"]
conv = []  # the metric matrix's conversion to numpy / Python (inside csv_ms)
_orig = decode._metrics_from_handle


def _timed(h):
    t0 = time.perf_counter()
    r = _orig(h)
    conv.append((time.perf_counter() - t0) * 1e3)
    return r


decode._metrics_from_handle = _timed
root = tempfile.mkdtemp(prefix="anomod_dec_")
d, mc, _ = bench._stage_tt_experiment((root, 0, bench.TT_FAULTS[0]))
js = next(str(p) for p in Path(d).glob("*.json"))
for th in threads:
    os.environ["ANOMOD_DECODE_THREADS"] = th
    out = {"threads": int(th), "json_mb": os.path.getsize(js) / 1e6,
           "csv_mb": os.path.getsize(mc) / 1e6}
    for name, fn in (("json_ms", lambda: decode.decode_native(decode.map_file(js), "skywalking")),
                     ("csv_ms", lambda: decode.decode_metric_long_csv_native(mc))):
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            fn()
            ts.append((time.perf_counter() - t0) * 1e3)
        out[name] = [round(x, 1) for x in ts]
    out["csv_conversion_ms"] = [round(x, 1) for x in conv[-5:]]
    print(json.dumps(out), flush=True)
