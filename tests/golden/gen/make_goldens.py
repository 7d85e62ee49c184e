#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ from the
REFERENCE's own code, run in this (survey/build) container.

The reference is only read at run time of this script — it is not imported
at module import and nothing of it is copied into the repo: only small
inputs and the outputs the reference computed from them are written.

  jaeger_small.json / jaeger_small.csv / jaeger_empty.csv
      synthetic Jaeger /api/traces dump -> SN_collection-scripts/Dataset/
      trace_data/jaeger_to_csv.py run as a subprocess (TZ=UTC)
  skywalking_small.json
      synthetic raw GraphQL span lists -> TT_collection-scripts/T-Dataset/
      trace_collector.py SkyWalkingTraceCollector._build_span_records
      (+ SpanRecord.to_dict, and a collector payload built from them)
  skywalking_dups.json
      raw GraphQL span lists whose duplicated node ids carry different parents
      (acyclic: a duplicate's parent was created before the node) ->
      _build_span_records; its BFS keeps the deepest visit of a node
  analyze_patterns.json
      synthetic ES segment hits -> enhanced_trace_collector.py
      extract_trace_info + analyze_trace_patterns
  percentiles.json
      latency lists -> SN .../api_responses/monitor_http_responses.py
      OpenAPIResponseCollector.generate_summary
  api_summary.json
      synthetic monitor responses -> SN .../api_responses/monitor_http_responses.py
      OpenAPIResponseCollector.generate_summary and enhanced_openapi_monitor.py
      EnhancedOpenAPIMonitor.generate_reports (the three report files; TZ=UTC)
  metric_long.csv / metric_results.json
      synthetic Prometheus query_range results -> TT_collection-scripts/
      T-Dataset/metric_collector.py MetricCollector.collect_experiment_metrics_csv
      (the HTTP query, boot-time probe and sleeps replaced by stubs; TZ=UTC)
  prom_dir/*.csv / prom_results.json
      synthetic Prometheus query_range results -> SN_collection-scripts/
      Dataset/metric_data/fetch_prometheus_metrics.py fetch_prometheus_metrics
      (requests.get stubbed) -> df.to_csv as its main() writes it (TZ=UTC)
  ewma_pandas.npz        pandas Series.ewm(alpha, adjust=False) mean/var
  pagerank_networkx.npz  networkx.pagerank (3.4.2, scipy backend)

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen/make_goldens.py [--only metric|api|swdup]
"""
from __future__ import annotations

import copy
import csv
import json
import os
import random
import subprocess
import sys
import tempfile
import types
from pathlib import Path

import numpy as np

REF = Path(os.environ.get("ANOMOD_REFERENCE", "/root/reference"))
OUT = Path(__file__).resolve().parents[1]
SN_SERVICES = ["compose-post-service", "home-timeline-service", "media-service",
               "nginx-web-server", "post-storage-service", "social-graph-service", "text-service",
               "unique-id-service", "url-shorten-service", "user-mention-service", "user-service",
               "user-timeline-service"]


def _hex(rng, n=16):
    return "".join(rng.choice("0123456789abcdef") for _ in range(n))


# ---------------------------------------------------------------------------
# Jaeger
# ---------------------------------------------------------------------------
def jaeger_doc(seed: int = 20251103, n_traces: int = 48) -> dict:
    rng = random.Random(seed)
    data = []
    for t in range(n_traces):
        tid = _hex(rng, 32 if t % 3 else 16)
        n_proc = rng.randint(1, 5)
        procs = {f"p{i + 1}": {"serviceName": rng.choice(SN_SERVICES), "tags": []}
                 for i in range(n_proc)}
        spans = []
        n = 0 if t == 5 else rng.randint(1, 14)
        ids = [_hex(rng) for _ in range(n)]
        if t == 7 and n > 2:
            ids[2] = ids[1]  # duplicate span id inside one trace
        for i in range(n):
            refs = []
            if i > 0:
                par = ids[rng.randrange(0, i)]
                kind = rng.random()
                if kind < 0.08:
                    refs = [{"refType": "FOLLOWS_FROM", "traceID": tid, "spanID": _hex(rng)},
                            {"refType": "CHILD_OF", "traceID": tid, "spanID": par}]
                elif kind < 0.14:
                    refs = [{"refType": "CHILD_OF", "traceID": tid, "spanID": par},
                            {"refType": "CHILD_OF", "traceID": tid, "spanID": ids[0]}]
                elif kind < 0.20:
                    refs = [{"refType": "CHILD_OF", "traceID": tid, "spanID": _hex(rng)}]  # orphan
                elif kind < 0.24:
                    refs = [{"refType": "FOLLOWS_FROM", "traceID": tid, "spanID": par}]
                else:
                    refs = [{"refType": "CHILD_OF", "traceID": tid, "spanID": par}]
            tags = [{"key": "component", "type": "string", "value": "thrift"}]
            r = rng.random()
            if r < 0.06:
                tags.append({"key": "error", "type": "bool", "value": True})
            elif r < 0.09:
                tags.append({"key": "http.status_code", "type": "int64", "value": 503})
            elif r < 0.12:
                tags.append({"key": "http.status_code", "type": "string", "value": "500"})
            elif r < 0.20:
                tags.append({"key": "http.status_code", "type": "int64", "value": 200})
                tags.append({"key": "http.method", "type": "string", "value": "GET"})
                tags.append({"key": "http.url", "type": "string", "value": "/wrk2-api/x"})
            elif r < 0.23:  # repeated key: last wins
                tags.append({"key": "error", "type": "bool", "value": True})
                tags.append({"key": "error", "type": "bool", "value": False})
            span = {
                "traceID": tid, "spanID": ids[i], "operationName": f"op_{rng.randint(0, 30)}",
                "references": refs,
                "startTime": 1762207200000000 + rng.randint(0, 3_600_000_000),
                "duration": rng.choice([0, 1, 63, 64, 65, 127, 128, 4095,
                                        rng.randint(1, 5_000_000)]),
                "tags": tags,
                "logs": ([{"timestamp": 1762207200000000 + rng.randint(0, 10**9),
                           "fields": [{"key": "event", "type": "string", "value": "x"}]}]
                         if rng.random() < 0.1 else []),
                "processID": rng.choice(list(procs)) if rng.random() > 0.03 else "p_missing",
            }
            if t == 11 and i == 0:
                del span["references"]
            spans.append(span)
        data.append({"traceID": tid, "spans": spans, "processes": procs, "warnings": None})
    return {"data": data, "total": 0, "limit": 0, "offset": 0, "errors": None}


def run_jaeger_to_csv(doc: dict, out_csv: Path) -> None:
    script = REF / "SN_collection-scripts/Dataset/trace_data/jaeger_to_csv.py"
    with tempfile.TemporaryDirectory() as td:
        inp = Path(td) / "in.json"
        inp.write_text(json.dumps(doc))
        env = dict(os.environ, TZ="UTC", PYTHONDONTWRITEBYTECODE="1")
        subprocess.run([sys.executable, str(script), str(inp), str(out_csv)], check=True,
                       env=env, cwd=td, capture_output=True)


# ---------------------------------------------------------------------------
# SkyWalking
# ---------------------------------------------------------------------------
def sw_traces(seed: int = 7, n_traces: int = 40) -> list[list[dict]]:
    rng = random.Random(seed)
    tt = ["ts-gateway-service", "ts-travel-service", "ts-route-service", "ts-order-service",
          "ts-basic-service", "ts-station-service", "ts-seat-service", "ts-auth-service"]
    out = []
    for t in range(n_traces):
        tid = f"{_hex(rng, 32)}.{rng.randint(1, 99)}.{rng.randint(10**15, 10**16)}"
        spans = []
        segs = []
        n_seg = rng.randint(1, 6)
        for s in range(n_seg):
            seg = _hex(rng, 32)
            svc = rng.choice(tt)
            n_sp = rng.randint(1, 5)
            parent_ref = None
            if s > 0:
                ps, pn = rng.choice(segs)
                parent_ref = {"traceId": tid, "parentSegmentId": ps,
                              "parentSpanId": rng.randrange(pn), "type": "CROSS_PROCESS"}
                if rng.random() < 0.1:
                    parent_ref["parentSegmentId"] = _hex(rng, 32)  # orphan: segment not in trace
                if rng.random() < 0.05:
                    parent_ref["parentSpanId"] = None
            for k in range(n_sp):
                st = 1762180000000 + rng.randint(0, 10**6)
                sp = {
                    "traceId": tid, "segmentId": seg, "spanId": k,
                    "parentSpanId": -1 if k == 0 else rng.randrange(k),
                    "serviceCode": svc, "serviceInstanceName": f"{svc}-pod",
                    "startTime": st, "endTime": st + rng.choice([0, 1, 2, 5, 17, 250, 3000, -3]),
                    "endpointName": f"/api/v1/{rng.randint(0, 9)}", "type": "Entry" if k == 0 else
                    rng.choice(["Exit", "Local"]), "peer": "", "component": "SpringMVC",
                    "isError": rng.random() < 0.1, "layer": "Http", "tags": [], "logs": [],
                    "refs": [parent_ref] if (k == 0 and parent_ref) else [],
                }
                spans.append(sp)
            segs.append((seg, n_sp))
        # edge cases
        if t == 3 and spans:
            del spans[-1]["segmentId"]
        if t == 4 and spans:
            spans[-1]["spanId"] = None
        if t == 5 and len(spans) > 1:
            spans.append(copy.deepcopy(spans[1]))  # duplicate node id
        if t == 6 and len(spans) > 1:
            spans[1]["parentSpanId"] = True  # bool is an int in the reference's test
        if t == 8 and spans:
            spans[0]["parentSpanId"] = None
        rng.shuffle(spans)  # GraphQL order is not tree order
        out.append(spans)
    return out


def sw_dup_traces(seed=13, n=60):
    """Traces where node ids repeat with different parents (the depth is the
    BFS's last = deepest visit).  Node k's parent and every duplicate's
    parent are drawn from nodes created before node k, so no cycle is
    reachable (the reference's BFS would not terminate)."""
    rng = random.Random(seed)
    out = []
    for t in range(n):
        tid = f"dup{t}"
        nodes = []  # (segment, span) in creation order
        spans = []
        big = t in (7, 31)
        n_nodes = rng.randint(200, 240) if big else rng.randint(2, 24)  # big: > 256 spans
        for k in range(n_nodes):
            seg = f"s{k // 3}"
            node = (seg, k % 3)
            parent = rng.randrange(k) if k and rng.random() < 0.95 else None
            nodes.append(node)
            copies = 1 + (rng.random() < 0.3) + (rng.random() < 0.1)
            for c in range(copies):
                p = parent if c == 0 else (rng.randrange(k) if k and rng.random() < 0.85 else None)
                if p is None:
                    ps, refs = -1, []
                elif nodes[p][0] == seg:
                    ps, refs = nodes[p][1], []
                else:
                    ps = -1
                    refs = [{"traceId": tid, "parentSegmentId": nodes[p][0],
                             "parentSpanId": nodes[p][1], "type": "CROSS_PROCESS"}]
                spans.append({"traceId": tid, "segmentId": seg, "spanId": node[1],
                              "parentSpanId": ps, "serviceCode": f"ts-s{rng.randint(0, 5)}-service",
                              "serviceInstanceName": "pod", "startTime": 1762180000000 + k,
                              "endTime": 1762180000000 + k + rng.randint(0, 50),
                              "endpointName": "/x", "type": "Local", "peer": "", "component": "x",
                              "isError": False, "layer": "Http", "tags": [], "logs": [],
                              "refs": refs})
        rng.shuffle(spans)
        out.append(spans)
    return out


def sw_expected(traces):
    sys.path.insert(0, str(REF / "TT_collection-scripts/T-Dataset"))
    try:
        import trace_collector as tc  # noqa: E402  (reference, run time only)
    finally:
        sys.path.pop(0)
    exp, payload_traces = [], []
    for spans in traces:
        recs, roots = tc.SkyWalkingTraceCollector._build_span_records(copy.deepcopy(spans))
        dicts = [r.to_dict() for r in recs]
        exp.append({
            "node_ids": [d["node_id"] for d in dicts],
            "parent_node_ids": [d["parent_node_id"] for d in dicts],
            "depths": [d["depth"] for d in dicts],
            "children": [d["children_node_ids"] for d in dicts],
            "duration_ms": [d["duration_ms"] for d in dicts],
            "is_error": [d["is_error"] for d in dicts],
            "service_code": [d["service_code"] for d in dicts],
            "roots": roots,
            "services_involved": sorted({r.service_code for r in recs if r.service_code}),
        })
        if recs:
            payload_traces.append({"summary": {"trace_id": recs[0].trace_id},
                                   "span_count": len(recs), "services_involved":
                                   exp[-1]["services_involved"], "root_span_node_ids": roots,
                                   "spans": dicts})
    return exp, {"metadata": {"generated_by": "reference _build_span_records"},
                 "traces": payload_traces}


# ---------------------------------------------------------------------------
# analyze_trace_patterns
# ---------------------------------------------------------------------------
def es_hits(seed=5, n=300):
    import base64
    rng = random.Random(seed)
    names = ["ts-order-service", "ts-travel-service", "ts-route-service", "ts-user-service"]
    hits = []
    for i in range(n):
        svc = rng.choice(names)
        sid = (base64.b64encode(svc.encode()).decode() + ".1") if rng.random() > 0.05 else ""
        st = 1762180000000 + rng.randint(0, 10**7) if rng.random() > 0.03 else 0
        hits.append({"_source": {
            "trace_id": _hex(rng, 32), "segment_id": _hex(rng, 32), "service_id": sid,
            "endpoint_name": rng.choice(["GET:/a", "POST:/b", "GET:/c", ""]),
            "start_time": st, "end_time": st + rng.randint(0, 3000),
            "latency": rng.choice([0, rng.randint(1, 5000), -1]),
            "is_error": rng.choice([0, 0, 0, 1]), "time_bucket": 0}})
    return {"hits": {"hits": hits}}


def analyze_expected(seg):
    sys.path.insert(0, str(REF / "TT_collection-scripts/T-Dataset"))
    try:
        import enhanced_trace_collector as etc_  # noqa: E402
    finally:
        sys.path.pop(0)
    cls = etc_.EnhancedTraceCollector
    traces = cls.extract_trace_info(None, copy.deepcopy(seg))
    res = cls.analyze_trace_patterns(None, traces)
    res["unique_services"] = sorted(res["unique_services"])
    res["unique_endpoints"] = sorted(res["unique_endpoints"])
    return traces, res


# ---------------------------------------------------------------------------
# percentiles (nearest rank)
# ---------------------------------------------------------------------------
def percentile_cases(seed=3):
    sys.path.insert(0, str(REF / "SN_collection-scripts/Dataset/api_responses"))
    try:
        import monitor_http_responses as mhr  # noqa: E402
    finally:
        sys.path.pop(0)
    rng = random.Random(seed)
    cases = []
    for n in [1, 2, 3, 7, 19, 20, 21, 99, 100, 101, 199, 200, 1000, 1001, 4999]:
        lat = [rng.randint(0, 63) if rng.random() < 0.6 else rng.randint(64, 10**6)
               for _ in range(n)]
        if n > 3:
            lat[0] = 0  # filtered by the reference's latency > 0 test
        ns = types.SimpleNamespace(
            responses=[{"status_code": 200, "latency_ms": v, "content_type": "application/json"}
                       for v in lat],
            start_time=0, duration=1, endpoints=["/x"])
        with tempfile.TemporaryDirectory() as td:
            p = Path(td) / "s.json"
            mhr.OpenAPIResponseCollector.generate_summary(ns, p)
            summ = json.loads(p.read_text())
        cases.append({"latencies": lat, "latency_statistics": summ["latency_statistics"]})
    return cases


# ---------------------------------------------------------------------------
# API-response monitors (generate_summary / generate_reports)
# ---------------------------------------------------------------------------
_EPS = ["/", "/wrk2-api/home-timeline/read", "/wrk2-api/user-timeline/read",
        "/wrk2-api/post/compose", "/wrk2-api/user/login"]
_CTYPES = ["application/json", "application/json; charset=utf-8", "text/html; charset=UTF-8",
           "text/plain", ""]


def api_responses(rng, n, int_latency=False):
    """Responses shaped as monitor_http_responses.py builds them (:62-111):
    ok responses with a rounded latency, timeouts (408 + 'error') and
    exceptions (status 0 + 'error'); some without content_type."""
    out, stats = [], {"total_requests": 0, "successful_requests": 0, "failed_requests": 0,
                      "status_codes": {}, "response_times": [], "errors": []}
    for _ in range(n):
        ep = rng.choice(_EPS)
        lat = rng.lognormvariate(3.0, 1.2)
        u = rng.random()
        if int_latency:
            lat = rng.randint(0, 2000) if rng.random() < 0.9 else 0
        if u < 0.06:
            r = {"endpoint": ep, "status_code": 408, "latency_ms": lat, "content_type": "",
                 "error": "timeout"}
            stats["errors"].append("timeout")
            stats["total_requests"] += 1
            stats["failed_requests"] += 1
        elif u < 0.09:
            r = {"endpoint": ep, "status_code": 0, "latency_ms": lat, "content_type": "",
                 "error": rng.choice(["Cannot connect", "Server disconnected"])}
            stats["errors"].append(r["error"])
            stats["total_requests"] += 1
            stats["failed_requests"] += 1
        else:
            code = rng.choice([200] * 12 + [201, 301, 302, 400, 404, 500, 502, 503])
            r = {"endpoint": ep, "status_code": code,
                 "latency_ms": lat if int_latency else round(lat, 2)}
            if rng.random() < 0.9:
                r["content_type"] = rng.choice(_CTYPES)
            stats["total_requests"] += 1
            stats["status_codes"][code] = stats["status_codes"].get(code, 0) + 1
            stats["response_times"].append(lat)
            if 200 <= code < 400:
                stats["successful_requests"] += 1
            else:
                stats["failed_requests"] += 1
        out.append(r)
    return out, stats


def api_goldens(seed=5):
    import logging
    d = REF / "SN_collection-scripts/Dataset/api_responses"
    sys.path.insert(0, str(d))
    try:
        import enhanced_openapi_monitor as eom  # noqa: E402
        import monitor_http_responses as mhr  # noqa: E402
    finally:
        sys.path.pop(0)
    rng = random.Random(seed)
    cases = []
    for n, int_lat in [(1, False), (2, True), (17, False), (64, True), (300, False),
                       (1000, False)]:
        responses, stats = api_responses(rng, n, int_lat)
        info = {"start_time": 1762128000.25 + n, "duration": 60 + n,
                "endpoints": _EPS[: 1 + n % 5], "sample_interval": 2}
        ns = types.SimpleNamespace(responses=responses, start_time=info["start_time"],
                                   duration=info["duration"], endpoints=info["endpoints"])
        with tempfile.TemporaryDirectory() as td:
            p = Path(td) / "s.json"
            mhr.OpenAPIResponseCollector.generate_summary(ns, p)
            summary = p.read_text()
        ens = types.SimpleNamespace(
            responses=responses, stats=copy.deepcopy(stats), start_time=info["start_time"],
            duration=info["duration"], endpoints=info["endpoints"],
            sample_interval=info["sample_interval"], logger=logging.getLogger("golden"))
        with tempfile.TemporaryDirectory() as td:
            ens.output_dir = Path(td)
            eom.EnhancedOpenAPIMonitor.generate_reports(ens)
            reports = {f: (Path(td) / f).read_text() for f in
                       ("response_summary.json", "status_code_distribution.csv",
                        "endpoint_performance.json")}
        cases.append({"responses": responses, "stats": stats, "info": info,
                      "summary_json": summary, "reports": reports})
    return cases


# ---------------------------------------------------------------------------
# pandas ewm / networkx pagerank
# ---------------------------------------------------------------------------
def ewma_golden(seed=11, T=600, S=6, alpha=2.0 / 61.0):
    import pandas as pd
    rng = np.random.default_rng(seed)
    X = (rng.uniform(-50, 1000, S) + rng.uniform(0.5, 5, S) * rng.standard_normal((T, S)))
    X = X.astype(np.float32)
    X[rng.random((T, S)) < 0.02] = np.nan
    X[:3, 1] = np.nan  # leading NaNs
    X[300:320, 2] += 40.0  # level shift
    M = np.empty((T, S))
    V = np.empty((T, S))
    for s in range(S):
        ser = pd.Series(X[:, s].astype(np.float64))
        e = ser.ewm(alpha=alpha, adjust=False, ignore_na=True)
        M[:, s] = e.mean().to_numpy()
        V[:, s] = e.var(bias=True).to_numpy()
    return {"X": X, "mean": M, "var": V, "alpha": np.float64(alpha)}


def pagerank_golden(seed=13, N=300, alpha=0.85):
    import networkx as nx
    rng = np.random.default_rng(seed)
    G = nx.DiGraph()
    G.add_nodes_from(range(N))
    for u in range(N):
        if rng.random() < 0.1:
            continue  # dangling
        for v in rng.choice(N, size=rng.integers(1, 12), replace=False):
            G.add_edge(int(u), int(v), weight=float(rng.integers(1, 1000)))
    p = rng.random(N)
    p[rng.random(N) < 0.5] = 0.0
    x = nx.pagerank(G, alpha=alpha, personalization={i: float(p[i]) for i in range(N)},
                    weight="weight", tol=1e-12, max_iter=1000)
    row_ptr = np.zeros(N + 1, np.uint32)
    col, w = [], []
    for u in range(N):
        nb = sorted(G.successors(u))
        col += nb
        w += [G[u][v]["weight"] for v in nb]
        row_ptr[u + 1] = len(col)
    return {"row_ptr": row_ptr, "col": np.asarray(col, np.uint32),
            "w": np.asarray(w, np.float32), "p": p, "alpha": np.float64(alpha),
            "x": np.asarray([x[i] for i in range(N)])}


# ---------------------------------------------------------------------------
# TT long-format metric CSV (metric_collector.py:400-478)
# ---------------------------------------------------------------------------
def prometheus_results(seed: int = 23) -> dict:
    """Synthetic query_range answers for a few of the collector's queries:
    several series per query, label sets that differ between series, 'NaN'
    samples, a query with no data (absent from the CSV) and a series without
    'metric' labels."""
    rng = random.Random(seed)
    t0 = 1762178400  # 2025-11-03 14:00:00 UTC
    pods = ["ts-order-service-7d9c", "ts-travel-service-5b8f", "ts-route-service-66a1"]

    def series(labels, n=12, nan_p=0.1, scale=1.0):
        vals = []
        for k in range(n):
            v = "NaN" if rng.random() < nan_p else repr(round(rng.uniform(0, 100) * scale, 6))
            vals.append([t0 + 15 * k, v])
        item = {"values": vals}
        if labels is not None:
            item["metric"] = labels
        return item

    res = {}
    res["rate(container_cpu_usage_seconds_total[1m])"] = [
        series({"__name__": "x", "namespace": "default", "pod": p, "container": p.rsplit("-", 1)[0]})
        for p in pods]
    res["container_memory_usage_bytes"] = [
        series({"pod": p, "namespace": "default"}, scale=1e6) for p in pods[:2]] + [
        series({"pod": pods[2], "instance": "10.0.0.7:9100", "job": "kubelet"}, scale=1e6)]
    res["up"] = [series({"job": "prometheus", "instance": "localhost:9090"}, nan_p=0.0),
                 series(None, n=5, nan_p=0.0)]
    res["process_open_fds"] = [series({"job": "node", "instance": "n1"}, n=8)]
    res["node_load1"] = []  # no data -> skipped by the collector
    return res


def metric_long_golden(results: dict, out_csv: Path) -> None:
    os.environ["TZ"] = "UTC"
    import time
    time.tzset()
    sys.path.insert(0, str(REF / "TT_collection-scripts/T-Dataset"))
    try:
        import metric_collector as mc  # noqa: E402  (reference, run time only)
    finally:
        sys.path.pop(0)
    import datetime as dt
    with tempfile.TemporaryDirectory() as tmp:
        col = mc.MetricCollector(prometheus_url="http://prometheus.invalid:9090", output_dir=tmp)
        col.key_metrics = list(results)

        def fake_range(self, query, start, end, step="15s"):
            r = results[query]
            return {"status": "success", "data": {"resultType": "matrix", "result": r}}

        col.query_prometheus_range = types.MethodType(fake_range, col)
        col.get_system_startup_time = types.MethodType(
            lambda self: dt.datetime(2025, 11, 3, 14, 0, 0), col)
        real_sleep = mc.time.sleep
        mc.time.sleep = lambda s: None
        try:
            path = col.collect_experiment_metrics_csv(experiment_name="golden", step="15s")
        finally:
            mc.time.sleep = real_sleep
        Path(out_csv).write_bytes(Path(path).read_bytes())


# ---------------------------------------------------------------------------
# SN metric directory (fetch_prometheus_metrics.py:9-80 + main :92-102,
# one CSV per query as collect_metric.sh:24-125 names them)
# ---------------------------------------------------------------------------
def sn_prometheus_results(seed: int = 31) -> dict:
    """Synthetic query_range answers for SN queries (file stem -> result
    list): several series per query with differing label sets, fractional
    timestamps, 'NaN' / '+Inf' / '-Inf' samples, tiny and huge values, a
    series with an empty label dict, label values holding commas and quotes,
    series of different lengths and offsets, and a no-data query (no file)."""
    rng = random.Random(seed)
    t0 = 1762207375.0  # 2025-11-03 22:02:55 UTC

    def values(n, start=0, frac=0.0, nan_p=0.05, scale=1.0, specials=()):
        out = []
        for k in range(n):
            ts = t0 + 15 * (start + k) + frac
            r = rng.random()
            if r < nan_p:
                v = "NaN"
            else:
                v = repr(round(rng.uniform(0, 100) * scale, 9))
            out.append([ts, v])
        for k, v in specials:
            out[k][1] = v
        return out

    svc = "container_label_com_docker_compose_service"
    res = {}
    res["socialnet_container_cpu"] = [
        {"metric": {svc: s}, "values": values(20, nan_p=0.1, scale=0.01)}
        for s in ("compose-post-service", "media-service", "user-timeline-service")]
    res["socialnet_container_memory"] = [
        {"metric": {"__name__": "container_memory_usage_bytes", svc: "post-storage-mongodb",
                    "container_label_com_docker_compose_project": "socialnetwork",
                    "id": "/docker/1f2e", "image": "mongo:4.4.6", "instance": "cadvisor:8080",
                    "job": "cadvisor", "name": "socialnetwork-post-storage-mongodb-1"},
         "values": values(20, scale=1e7, specials=((3, "+Inf"), (4, "-Inf")))},
        {"metric": {"__name__": "container_memory_usage_bytes", svc: "text-service",
                    "instance": "cadvisor:8080", "job": "cadvisor"},
         "values": values(12, start=5, scale=1e7)},
    ]
    # fractional timestamps (a window not aligned to whole seconds)
    res["socialnet_container_network_receive"] = [
        {"metric": {svc: "nginx-thrift"}, "values": values(16, frac=0.5, scale=1e3)},
        {"metric": {svc: "home-timeline-service"}, "values": values(16, frac=0.5, nan_p=0.3)},
    ]
    # an aggregate without labels ('metric' = '') and label values with
    # commas and quotes
    res["mongodb_operations_rate"] = [
        {"metric": {}, "values": values(10, scale=1e-6)},
        {"metric": {"type": "query,insert", "note": 'say "hi"'}, "values": values(10, start=3)},
    ]
    res["microservice_request_rate"] = []  # no data -> no file (fetch_prometheus_metrics.py:101-102)
    return res


def sn_prometheus_golden(results: dict, out_dir: Path) -> None:
    """Run the reference fetch_prometheus_metrics() with requests.get stubbed
    and write each DataFrame as its main() does (df.to_csv(index=False))."""
    os.environ["TZ"] = "UTC"
    import time
    time.tzset()
    sys.path.insert(0, str(REF / "SN_collection-scripts/Dataset/metric_data"))
    try:
        import fetch_prometheus_metrics as fpm  # noqa: E402  (reference, run time only)
    finally:
        sys.path.pop(0)

    class _Resp:
        def __init__(self, payload):
            self.payload = payload

        def raise_for_status(self):
            return None

        def json(self):
            return self.payload

    current = {}

    def fake_get(url, params=None, **kw):
        return _Resp({"status": "success",
                      "data": {"resultType": "matrix", "result": current["result"]}})

    out_dir.mkdir(parents=True, exist_ok=True)
    for old in out_dir.glob("*.csv"):
        old.unlink()
    real_requests = fpm.requests
    fpm.requests = types.SimpleNamespace(get=fake_get, exceptions=real_requests.exceptions)
    try:
        for stem, result in results.items():
            current["result"] = result
            df = fpm.fetch_prometheus_metrics(stem, int(t0_of(result)), int(t0_of(result)) + 3600,
                                              "15s", "http://prometheus.invalid:9090")
            if df is not None:
                df.to_csv(out_dir / f"{stem}.csv", index=False)
    finally:
        fpm.requests = real_requests


def t0_of(result) -> float:
    return min((v[0][0] for r in result for v in [r["values"]] if v), default=0.0)


def main():
    OUT.mkdir(parents=True, exist_ok=True)
    only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
    if only in (None, "prom"):
        res = sn_prometheus_results()
        (OUT / "prom_results.json").write_text(json.dumps(res))
        sn_prometheus_golden(res, OUT / "prom_dir")
    if only in (None, "metric"):
        res = prometheus_results()
        (OUT / "metric_results.json").write_text(json.dumps(res))
        metric_long_golden(res, OUT / "metric_long.csv")
    if only in (None, "api"):
        (OUT / "api_summary.json").write_text(json.dumps(api_goldens()))
    if only in (None, "swdup"):
        dups = sw_dup_traces()
        dexp, _ = sw_expected(dups)
        (OUT / "skywalking_dups.json").write_text(json.dumps({"inputs": dups, "expected": dexp}))
    if only is not None:
        return
    doc = jaeger_doc()
    (OUT / "jaeger_small.json").write_text(json.dumps(doc))
    run_jaeger_to_csv(doc, OUT / "jaeger_small.csv")
    run_jaeger_to_csv({"data": []}, OUT / "jaeger_empty.csv")

    traces = sw_traces()
    expected, payload = sw_expected(traces)
    (OUT / "skywalking_small.json").write_text(json.dumps(
        {"inputs": traces, "expected": expected, "payload": payload}))

    seg = es_hits()
    tr, res = analyze_expected(seg)
    (OUT / "analyze_patterns.json").write_text(json.dumps(
        {"segments": seg, "traces": tr, "analysis": res}, default=str))

    (OUT / "percentiles.json").write_text(json.dumps(percentile_cases()))
    np.savez_compressed(OUT / "ewma_pandas.npz", **ewma_golden())
    np.savez_compressed(OUT / "pagerank_networkx.npz", **pagerank_golden())
    import networkx
    import pandas
    (OUT / "VERSIONS.json").write_text(json.dumps({
        "python": sys.version.split()[0], "pandas": pandas.__version__,
        "networkx": networkx.__version__, "numpy": np.__version__,
        "reference": str(REF), "TZ": "UTC"}, indent=2))
    print("goldens written to", OUT)


if __name__ == "__main__":
    main()
