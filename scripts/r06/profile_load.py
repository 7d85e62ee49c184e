#!/usr/bin/env python3
"""Where load_experiment spends a config-2 experiment read from files (host
only): the trace payload and the metric CSV decoded on two threads
(engine.load_experiment), each also timed alone; 5 loads after one warm-up.

  python scripts/r06/profile_load.py"""
import json
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"), str(ROOT)]

import anomod  # noqa: E402
import bench  # noqa: E402
from anomod import decode  # noqa: E402

d, mc, _ = bench._stage_tt_experiment((tempfile.mkdtemp(prefix="anomod_load_"), 0, bench.TT_FAULTS[0]))
js = next(Path(d).glob("*.json"))
anomod.load_experiment(d, metrics=mc)


def t(f, n=5):
    out = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        out.append(round((time.perf_counter() - t0) * 1e3, 1))
    return out


print(json.dumps({"load_experiment_ms": t(lambda: anomod.load_experiment(d, metrics=mc)),
                  "trace_file_ms": t(lambda: decode.load_trace_file(js)),
                  "trace_decode_only_ms": t(lambda: decode.decode_native(decode.map_file(js),
                                                                         "skywalking")),
                  "metric_csv_ms": t(lambda: decode.decode_metric_long_csv_native(mc))}))
