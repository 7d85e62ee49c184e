#!/usr/bin/env python3
"""Where a host set's first Context.edge_aggregate call goes (LONG, 2^20
traces, 55.6 M spans): the same SpanSet uploaded alone (anomod_spans_upload)
and aggregated through the host path, first and later calls, each timed on
its own; a second, never-seen copy of the arrays isolates first-touch
registration costs.

  python scripts/r06/first_host_call.py"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"), str(ROOT)]

import numpy as np  # noqa: E402

import anomod  # noqa: E402


def ms(f):
    t0 = time.perf_counter()
    r = f()
    return (time.perf_counter() - t0) * 1e3, r


with anomod.Context(0) as ctx:
    lh = ctx.generate(anomod.SynthSpec("LONG", seed=20251106, p_orphan_ppm=100), 1 << 20)
    host = lh.download()
    lh.free()
    out = {"spans": host.n_spans}
    if "--warm" in sys.argv:  # a 1.1 M-span set first (8-MiB+ columns: the registered path)
        wh = ctx.generate(anomod.SynthSpec("SN", seed=7), 1 << 17)
        small = wh.download()
        wh.free()
        t, d = ms(lambda: ctx.upload(small))
        out["warm_upload_ms"] = t
        out["warm_spans"] = small.n_spans
        d.free()
    t, dev = ms(lambda: ctx.upload(host))
    out["upload_first_ms"] = t
    dev.free()
    t, dev = ms(lambda: ctx.upload(host))
    out["upload_second_ms"] = t
    dev.free()
    out["aggregate_ms"] = [ms(lambda: ctx.edge_aggregate(host, with_hist=True))[0] for _ in range(3)]
    copy = anomod.SpanSet(host.services, host.trace_ptr.copy(), host.trace_hash.copy(),
                          host.span_id.copy(), host.parent_span_id.copy(), host.svc.copy(),
                          host.flags.copy(), host.dur_us.copy())
    out["aggregate_fresh_copy_ms"] = [ms(lambda: ctx.edge_aggregate(copy, with_hist=True))[0]
                                      for _ in range(2)]
    print(json.dumps({k: (np.round(v, 1).tolist() if isinstance(v, list) else
                          round(v, 1) if isinstance(v, float) else v) for k, v in out.items()}))
