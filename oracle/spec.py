"""Pure-Python / numpy restatement of the reference's per-span rules
(TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

Written independently of the product decoders in anomod/decode.py so the two
can be checked against each other and against the reference goldens.
"""
from __future__ import annotations

import math
from collections import deque
from datetime import datetime

import numpy as np


# ---- SN / Jaeger: jaeger_to_csv.py:21-90 ---------------------------------
def jaeger_rows(doc: dict) -> list[dict]:
    rows = []
    for trace in doc.get("data", []):                                   # :21
        tid = trace.get("traceID", "")                                   # :22
        p2s = {k: v.get("serviceName", "") for k, v in trace.get("processes", {}).items()}
        for span in trace.get("spans", []):                              # :32
            parent = ""
            for ref in span.get("references", []):                       # :35-38
                if ref.get("refType") == "CHILD_OF":
                    parent = ref.get("spanID", "")
                    break
            tags = {}
            for tag in span.get("tags", []):                             # :55-58
                tags[tag.get("key", "")] = tag.get("value", "")
            rows.append({"trace_id": tid, "span_id": span.get("spanID", ""),
                         "parent_span_id": parent,
                         "service": p2s.get(span.get("processID", ""), ""),  # :45-46
                         "duration_us": span.get("duration", 0), "tags": tags})  # :83
    return rows


# ---- TT / SkyWalking: trace_collector.py:401-481 ---------------------------
def build_span_records(spans: list[dict]):
    """node ids, parent node ids, children, depth (BFS from roots), roots."""
    nodes, parents, children, order = {}, {}, {}, []
    for span in spans:                                                   # :409-417
        seg, sid = span.get("segmentId"), span.get("spanId")
        if seg is None or sid is None:
            order.append(None)
            continue
        nid = f"{seg}:{sid}"
        order.append(nid)
        nodes[nid] = span
        children.setdefault(nid, [])
    for span, nid in zip(spans, order):                                  # :420-439
        if nid is None:
            continue
        pn = None
        psid = span.get("parentSpanId", -1)
        if isinstance(psid, int) and psid >= 0:
            pn = f"{span.get('segmentId')}:{psid}"
        else:
            refs = span.get("refs") or []
            if refs:
                ps, pp = refs[0].get("parentSegmentId"), refs[0].get("parentSpanId")
                if ps is not None and pp is not None:
                    pn = f"{ps}:{pp}"
        parents[nid] = pn
        if pn and pn in children:
            children[pn].append(nid)
    depth = {}
    roots = [n for n, p in parents.items() if p not in nodes]            # :443
    q = deque((n, 0) for n in roots)
    while q:                                                             # :445-449
        cur, d = q.popleft()
        depth[cur] = d
        for ch in children.get(cur, []):
            q.append((ch, d + 1))
    recs = []
    for span, nid in zip(spans, order):                                  # :452-479
        if nid is None:
            continue
        recs.append({"node_id": nid, "parent_node_id": parents.get(nid),
                     "children": list(children.get(nid, [])), "depth": depth.get(nid, 0),
                     "duration_ms": max(0, span.get("endTime", 0) - span.get("startTime", 0)),
                     "is_error": bool(span.get("isError", False)),
                     "service_code": span.get("serviceCode")})
    return recs, roots


# ---- enhanced_trace_collector.py:216-296 ----------------------------------
def analyze_trace_patterns(traces: list[dict]) -> dict:
    if not traces:
        return {"total_traces": 0, "unique_services": [], "unique_endpoints": [],
                "error_traces": 0, "service_call_counts": {}, "endpoint_call_counts": {},
                "latency_stats": None, "time_range": {"earliest": None, "latest": None}}
    svc_c, ep_c, lat, err = {}, {}, [], 0
    lo = hi = None
    for t in traces:
        s = t.get("service_name", "unknown")
        svc_c[s] = svc_c.get(s, 0) + 1
        e = t.get("endpoint_name", "unknown")
        ep_c[e] = ep_c.get(e, 0) + 1
        if t.get("is_error", 0) == 1:
            err += 1
        if t.get("latency", 0) > 0:
            lat.append(t["latency"])
        st = t.get("start_time", 0)
        if st:
            lo = st if lo is None or st < lo else lo
            hi = st if hi is None or st > hi else hi
    stats = ({"min": min(lat), "max": max(lat), "avg": sum(lat) / len(lat), "count": len(lat)}
             if lat else [])
    return {"total_traces": len(traces), "unique_services": sorted(svc_c),
            "unique_endpoints": sorted(ep_c), "error_traces": err,
            "service_call_counts": svc_c, "endpoint_call_counts": ep_c, "latency_stats": stats,
            "time_range": {"earliest": lo, "latest": hi}}


# ---- monitor_http_responses.py:180-190 ------------------------------------
def nearest_rank(values, q_pct: int):
    v = sorted(values)
    return v[len(v) * q_pct // 100]


# ---- monitor_http_responses.py:150-207 / enhanced_openapi_monitor.py:318-393
def latency_picks(values: list, suffix: str = "") -> dict:
    """min / max / mean / median / p95 / p99 of a sorted copy (:180-190)."""
    if not values:
        return {}
    v = sorted(values)
    n = len(v)
    return {"min" + suffix: v[0], "max" + suffix: v[-1], "mean" + suffix: sum(v) / n,
            "median" + suffix: v[n // 2], "p95" + suffix: v[int(n * 0.95)],
            "p99" + suffix: v[int(n * 0.99)]}


def response_summary(responses: list[dict], start_time, duration, endpoints):
    """generate_summary's dict (:150-205); None for no responses."""
    if not responses:
        return None
    codes, ctypes_, lat, err = {}, {}, [], 0
    for r in responses:
        c = r.get("status_code", 0)
        codes[c] = codes.get(c, 0) + 1
        x = r.get("latency_ms", 0)
        if x > 0:
            lat.append(x)
        t = r.get("content_type", "unknown").split(";")[0]
        ctypes_[t] = ctypes_.get(t, 0) + 1
        err += "error" in r
    n = len(responses)
    return {"collection_info": {"start_time": datetime.fromtimestamp(start_time).isoformat(),
                                "duration_seconds": duration, "total_responses": n,
                                "endpoints_monitored": endpoints},
            "status_code_distribution": codes, "latency_statistics": latency_picks(lat),
            "content_type_distribution": ctypes_, "error_count": err,
            "success_rate": (n - err) / n * 100}


def response_reports(responses, stats, start_time, duration, endpoints, sample_interval):
    """generate_reports' three outputs (:318-393): summary dict, CSV text,
    endpoint-performance dict."""
    codes = dict(stats["status_codes"])
    summary = {
        "collection_info": {"start_time": datetime.fromtimestamp(start_time).isoformat(),
                            "duration_seconds": duration, "total_responses": len(responses),
                            "endpoints_monitored": endpoints,
                            "sample_interval_seconds": sample_interval},
        "statistics": {"total_requests": stats["total_requests"],
                       "successful_requests": stats["successful_requests"],
                       "failed_requests": stats["failed_requests"],
                       "success_rate_percent": (stats["successful_requests"]
                                                / max(1, stats["total_requests"])) * 100},
        "status_code_distribution": codes,
        "latency_statistics": latency_picks(stats["response_times"], "_ms"),
        "error_summary": {"total_errors": len(stats["errors"]),
                          "unique_errors": len(set(stats["errors"])),
                          "common_errors": list(set(stats["errors"]))}}
    total = sum(codes.values())
    csv_text = "status_code,count,percentage\n" + "".join(
        f"{c},{k},{(k / total * 100) if total > 0 else 0:.2f}\n" for c, k in sorted(codes.items()))
    perf: dict = {}
    for r in responses:
        e = perf.setdefault(r.get("endpoint", "unknown"),
                            {"count": 0, "avg_latency": 0, "status_codes": {}})
        e["count"] += 1
        e["avg_latency"] += r.get("latency_ms", 0)
        st = r.get("status_code", 0)
        e["status_codes"][st] = e["status_codes"].get(st, 0) + 1
    for e in perf.values():
        e["avg_latency"] /= e["count"]
    return summary, csv_text, perf


# ---- histogram binning (build-defined, include/anomod.h) ------------------
def hist_bin(v: int) -> int:
    if v < 64:
        return v
    e = v.bit_length() - 1 - 5
    return (e << 5) + (v >> e)


def hist_bounds(b: int) -> tuple[int, int]:
    if b < 64:
        return b, b
    e = (b >> 5) - 1
    m = (b & 31) + 32
    return m << e, ((m + 1) << e) - 1


def edge_table_py(spans, S: int) -> dict:
    """Pure-Python edge table for tiny span sets (first match in trace order)."""
    E = (S + 2) * S
    out = {"count": [0] * E, "errors": [0] * E, "sum_us": [0] * E,
           "min_us": [0xFFFFFFFF] * E, "max_us": [0] * E, "hist": {}}
    for t in range(spans.n_traces):
        a, b = int(spans.trace_ptr[t]), int(spans.trace_ptr[t + 1])
        for i in range(a, b):
            pid = int(spans.parent_span_id[i])
            p = S
            if pid:
                p = S + 1
                for q in range(a, b):
                    if int(spans.span_id[q]) == pid:
                        p = int(spans.svc[q])
                        break
            e = p * S + int(spans.svc[i])
            d = int(spans.dur_us[i])
            out["count"][e] += 1
            out["errors"][e] += int(spans.flags[i]) & 1
            out["sum_us"][e] += d
            out["min_us"][e] = min(out["min_us"][e], d)
            out["max_us"][e] = max(out["max_us"][e], d)
            k = (e, hist_bin(d))
            out["hist"][k] = out["hist"].get(k, 0) + 1
    return out


# ---- EWMA / z-score (build-defined; pandas ewm adjust=False) --------------
def ewma_state(x: np.ndarray, alpha: float):
    """Per-step (m, v) of one series, NaN samples skipped (ignore_na=True)."""
    m = np.full(x.shape[0], np.nan)
    v = np.full(x.shape[0], np.nan)
    cm = cv = None
    for t, xv in enumerate(x.astype(np.float64)):
        if not math.isnan(xv):
            if cm is None:
                cm, cv = xv, 0.0
            else:
                d = xv - cm
                cm = cm + alpha * d
                cv = (1 - alpha) * (cv + alpha * d * d)
        if cm is not None:
            m[t], v[t] = cm, cv
    return m, v


def window_scores_from_state(X: np.ndarray, M: np.ndarray, V: np.ndarray, W: int,
                             eps: float) -> np.ndarray:
    """Z[w, s] = max |z_t| over window w, z_t = (x_t - m_{t-1})/sqrt(v_{t-1}+eps)."""
    T, S = X.shape
    Z = np.zeros((T // W, S))
    for s in range(S):
        seen = False
        for t in range(T):
            x = float(X[t, s])
            z = 0.0
            if not math.isnan(x):
                if seen:
                    z = (x - M[t - 1, s]) / math.sqrt(V[t - 1, s] + eps)
                seen = True
            # carry state across NaNs: M/V at t-1 already hold the last state
            Z[t // W, s] = max(Z[t // W, s], abs(z))
    return Z


# ---- ungrouped span sets: the grouping rule of anomod_spans_group ----------
# (no reference counterpart: the reference's collectors hand spans over per
# trace, trace_collector.py:539-546; the ES path enhanced_trace_collector.py:
# 80-90,109-110 pulls hits sorted by start_time across traces)
def mix64(h) -> np.ndarray:
    """SplitMix64 finaliser (a bijection of u64), elementwise."""
    z = np.array(h, dtype=np.uint64, copy=True).reshape(-1)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def group_by_trace(trace_hash) -> tuple[np.ndarray, np.ndarray]:
    """(order, trace_ptr): spans taken in `order` are grouped by trace —
    traces by mix64(trace_hash) ascending, spans of a trace in arrival order
    (a stable sort)."""
    k = mix64(trace_hash)
    order = np.argsort(k, kind="stable")
    ks = k[order]
    n = ks.shape[0]
    starts = np.flatnonzero(np.r_[True, ks[1:] != ks[:-1]]) if n else np.zeros(0, np.int64)
    return order, np.r_[starts, n].astype(np.uint64)


# ---- long traces with unique span ids: vectorised restatement -------------
# The C oracle resolves parents by an ordered scan, O(L^2) per trace — minutes
# for a 10^5-span trace.  When every id is unique inside its trace, the first
# match of a parent reference is its only match, so a sorted-id lookup gives
# the same parents (jaeger_to_csv.py:34-38, trace_collector.py:424-443), and
# the BFS depth of _build_span_records (:441-449) is the length of the parent
# chain up to a root (0 when the chain never reaches one: a cycle).
def hist_bins_np(d) -> np.ndarray:
    """hist_bin over a u32 array."""
    v = np.asarray(d, np.uint64)
    bl = np.zeros(v.shape, np.uint64)
    for k in range(32):
        bl += (v >> np.uint64(k)) > 0
    e = np.where(v < 64, np.uint64(0), bl - np.uint64(6))
    return np.where(v < 64, v, (e << np.uint64(5)) + (v >> e)).astype(np.int64)


def unique_id_parents(spans) -> np.ndarray:
    """Trace-local parent position of every span (-1: parent reference 0 or
    not in the trace), for span sets whose ids are unique inside each trace."""
    ptr = np.asarray(spans.trace_ptr, np.int64)
    n = int(ptr[-1]) if ptr.size else 0
    lens = np.diff(ptr)
    t_of = np.repeat(np.arange(lens.size), lens)
    sid = np.asarray(spans.span_id, np.uint64)[:n]
    pid = np.asarray(spans.parent_span_id, np.uint64)[:n]
    order = np.lexsort((sid, t_of))  # by (trace, id)
    key_t, key_id = t_of[order], sid[order]
    assert not np.any((key_t[1:] == key_t[:-1]) & (key_id[1:] == key_id[:-1])), \
        "ids repeat inside a trace: use the C oracle"
    # per-span binary search of its parent reference inside its trace's id run
    lo = np.searchsorted(key_t, t_of, "left")
    hi = np.searchsorted(key_t, t_of, "right")
    out = np.full(n, -1, np.int64)
    idx = np.zeros(n, np.int64)
    for t in range(lens.size):
        a, b = int(ptr[t]), int(ptr[t + 1])
        if a == b:
            continue
        r0, r1 = int(lo[a]), int(hi[a])
        j = np.searchsorted(key_id[r0:r1], pid[a:b]) + r0
        idx[a:b] = np.minimum(j, r1 - 1)
    found = (pid != 0) & (key_id[idx] == pid) & (key_t[idx] == t_of)
    out[found] = order[idx[found]] - ptr[t_of[found]]
    return out


def unique_id_edge_table(spans, S: int) -> dict:
    """Edge table (as oracle_edge_aggregate) for unique-id span sets."""
    ptr = np.asarray(spans.trace_ptr, np.int64)
    n = int(ptr[-1]) if ptr.size else 0
    par = unique_id_parents(spans)
    svc = np.asarray(spans.svc, np.int64)[:n]
    t_of = np.repeat(np.arange(ptr.size - 1), np.diff(ptr))
    pid = np.asarray(spans.parent_span_id, np.uint64)[:n]
    p = np.where(pid == 0, S, S + 1)
    has = par >= 0
    p[has] = svc[ptr[t_of[has]] + par[has]]
    e = p * S + svc
    E = (S + 2) * S
    d = np.asarray(spans.dur_us, np.uint32)[:n]
    err = (np.asarray(spans.flags, np.int64)[:n] & 1).astype(bool)
    tab = {"count": np.bincount(e, minlength=E).astype(np.uint64),
           "errors": np.bincount(e[err], minlength=E).astype(np.uint64),
           "sum_us": np.zeros(E, np.uint64), "min_us": np.full(E, 0xFFFFFFFF, np.uint32),
           "max_us": np.zeros(E, np.uint32)}
    np.add.at(tab["sum_us"], e, d.astype(np.uint64))
    np.minimum.at(tab["min_us"], e, d)
    np.maximum.at(tab["max_us"], e, d)
    tab["hist"] = np.bincount(e * 896 + hist_bins_np(d), minlength=E * 896).astype(
        np.uint64).reshape(E, 896)
    tab["edge"] = e
    return tab


def unique_id_trace_structure(spans, S: int) -> dict:
    """oracle_trace_structure's outputs for unique-id span sets."""
    ptr = np.asarray(spans.trace_ptr, np.int64)
    nt = ptr.size - 1
    n = int(ptr[-1]) if ptr.size else 0
    par = unique_id_parents(spans)
    t_of = np.repeat(np.arange(nt), np.diff(ptr))
    gpar = np.where(par >= 0, par + ptr[t_of], -1)  # global parent index
    svc = np.asarray(spans.svc, np.int64)[:n]
    words = (S + 63) // 64
    root = par < 0
    # depth: pointer jumping up the parent chain (kDone = reached a root)
    nxt = np.where(root, np.arange(n), gpar)
    dst = np.where(root, 0, 1).astype(np.int64)
    done = root.copy()
    for _ in range(64):
        if done.all():
            break
        live = ~done
        dst[live] += dst[nxt[live]]
        done_n = done.copy()
        done_n[live] = done[nxt[live]]
        nxt[live] = nxt[nxt[live]]
        done = done_n
    mask = np.zeros((nt, words), np.uint64)
    np.bitwise_or.at(mask, (t_of, svc >> 6), np.left_shift(np.uint64(1), (svc & 63).astype(np.uint64)))
    return {"parent_pos": np.where(root, 0xFFFFFFFF, par).astype(np.uint32),
            "depth": np.where(done, dst, 0).astype(np.uint32),
            "n_children": np.bincount(gpar[gpar >= 0], minlength=n).astype(np.uint32),
            "span_flags": np.where(root, 3, 2).astype(np.uint8),
            "n_roots": np.bincount(t_of[root], minlength=nt).astype(np.uint32),
            "svc_mask": mask}
