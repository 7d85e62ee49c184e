#!/usr/bin/env python3
"""Decode throughput on a synthetic Jaeger dump shaped like SN_data's
all_traces.json (pretty-printed like the jq merge, ~10 spans per trace):
native decoder (libanomod) vs the Python json.load + per-span decoder."""
import json
import random
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"), str(ROOT)]
import anomod  # noqa: E402
from anomod import decode  # noqa: E402


def doc(n_traces, seed=1):
    rng = random.Random(seed)
    svcs = ["compose-post-service", "home-timeline-service", "media-service", "nginx-web-server",
            "post-storage-service", "social-graph-service", "text-service", "user-service"]
    data = []
    for _ in range(n_traces):
        tid = "%032x" % rng.getrandbits(128)
        ids = ["%016x" % rng.getrandbits(64) for _ in range(10)]
        spans = []
        for j, sid in enumerate(ids):
            spans.append({
                "traceID": tid, "spanID": sid, "flags": 1, "operationName": f"op_{j}",
                "references": ([{"refType": "CHILD_OF", "traceID": tid, "spanID": ids[j // 2]}]
                               if j else []),
                "startTime": 1762207158839501 + j * 37, "duration": rng.randint(10, 90000),
                "tags": [{"key": "component", "type": "string", "value": "thrift"},
                         {"key": "internal.span.format", "type": "string", "value": "proto"}],
                "logs": [], "processID": f"p{j % 4 + 1}", "warnings": None})
        procs = {f"p{k}": {"serviceName": rng.choice(svcs),
                           "tags": [{"key": "hostname", "type": "string", "value": "h"}]}
                 for k in range(1, 5)}
        data.append({"traceID": tid, "spans": spans, "processes": procs, "warnings": None})
    return {"data": data, "total": 0, "limit": 0, "offset": 0, "errors": None}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    raw = json.dumps(doc(n), indent=2).encode()
    t0 = time.perf_counter()
    nat = anomod.decode_native(raw, "jaeger")
    t1 = time.perf_counter()
    py = decode.decode_jaeger(json.loads(raw))
    t2 = time.perf_counter()
    assert (nat.span_id == py.span_id).all() and (nat.svc == py.svc).all()
    print(json.dumps({"bytes": len(raw), "spans": nat.n_spans,
                      "native_s": t1 - t0, "native_MBps": len(raw) / (t1 - t0) / 1e6,
                      "native_spans_per_s": nat.n_spans / (t1 - t0),
                      "python_s": t2 - t1, "python_spans_per_s": py.n_spans / (t2 - t1),
                      "speedup": (t2 - t1) / (t1 - t0)}))


if __name__ == "__main__":
    main()
