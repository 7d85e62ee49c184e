"""SkyWalking segment records (Elasticsearch ``sw_segment-*`` hits) and their
summary — the drop-in for EnhancedTraceCollector.extract_trace_info +
analyze_trace_patterns (TT_collection-scripts/T-Dataset/
enhanced_trace_collector.py:102-165, 216-296).

Decoding (service name from the base64 service id, field defaults) is host
work restated from the reference; the summary itself — counts per service
and endpoint, error count, latency and time-range reductions — runs in the
segment-summary HIP kernel (libanomod ``anomod_segment_summary``).
"""
from __future__ import annotations

import base64
import ctypes as C
import datetime
from dataclasses import dataclass

import numpy as np

from . import _lib as L


def service_name_of(service_id) -> str:
    """extract_trace_info's service-name decoding (:130-150): the base64 part
    before the first '.', decoded as UTF-8, else that part as plain text;
    'unknown' when the id is empty."""
    if not service_id:
        return "unknown"
    try:
        part = service_id.split(".")[0]
        try:
            return base64.b64decode(part).decode("utf-8")
        except Exception:  # noqa: BLE001 — the reference's bare except (:143)
            return part
    except Exception:  # noqa: BLE001 (:146)
        return service_id


def trace_infos(segment_data) -> list[dict]:
    """The per-hit dicts extract_trace_info builds (:102-165), without the
    ISO datetime strings it adds for display."""
    if not segment_data or "hits" not in segment_data:
        return []
    out = []
    for hit in segment_data["hits"]["hits"]:
        src = hit["_source"]
        info = {
            "trace_id": src.get("trace_id", ""), "segment_id": src.get("segment_id", ""),
            "service_id": src.get("service_id", ""),
            "endpoint_name": src.get("endpoint_name", ""),
            "start_time": src.get("start_time", 0), "end_time": src.get("end_time", 0),
            "latency": src.get("latency", 0), "is_error": src.get("is_error", 0),
        }
        info["service_name"] = service_name_of(info["service_id"])
        out.append(info)
    return out


@dataclass
class SegmentSet:
    """Columnar segment records.  ``services`` / ``endpoints`` list the names
    in first-appearance order (the insertion order of the reference's
    count dicts); ``svc`` / ``endpoint`` index them."""

    services: list[str]
    endpoints: list[str]
    svc: np.ndarray        # u32 [n]
    endpoint: np.ndarray   # u32 [n]
    is_error: np.ndarray   # i32 [n]  1 exactly when the record's is_error == 1
    latency: np.ndarray    # i64 [n]
    start_time: np.ndarray  # i64 [n]

    @property
    def n(self) -> int:
        return int(self.svc.shape[0])

    @staticmethod
    def from_traces(traces: list[dict]) -> "SegmentSet":
        """From extract_trace_info-style dicts (the input of
        analyze_trace_patterns); missing keys take that function's defaults."""
        svc_idx: dict[str, int] = {}
        ep_idx: dict[str, int] = {}
        n = len(traces)
        svc = np.empty(n, np.uint32)
        ep = np.empty(n, np.uint32)
        err = np.empty(n, np.int32)
        lat = np.empty(n, np.int64)
        st = np.empty(n, np.int64)
        for i, t in enumerate(traces):
            s = t.get("service_name", "unknown")
            e = t.get("endpoint_name", "unknown")
            svc[i] = svc_idx.setdefault(s, len(svc_idx))
            ep[i] = ep_idx.setdefault(e, len(ep_idx))
            err[i] = 1 if t.get("is_error", 0) == 1 else 0
            lat[i] = int(t.get("latency", 0) or 0)
            st[i] = int(t.get("start_time", 0) or 0)
        return SegmentSet(list(svc_idx), list(ep_idx), svc, ep, err, lat, st)

    @staticmethod
    def from_es(segment_data) -> "SegmentSet":
        return SegmentSet.from_traces(trace_infos(segment_data))


def _iso_ms(ms: int) -> str:
    return datetime.datetime.fromtimestamp(ms / 1000).isoformat()


def segment_summary(ctx, seg: SegmentSet) -> dict:
    """analyze_trace_patterns' result dict (:216-296) computed on the GPU.
    ``unique_*`` lists are sorted (the reference's come from a set, so their
    order is arbitrary); count dicts keep first-appearance order."""
    if seg.n == 0:  # the reference's early return (:218-228)
        return {"total_traces": 0, "unique_services": [], "unique_endpoints": [],
                "error_traces": 0, "service_call_counts": {}, "endpoint_call_counts": {},
                "latency_stats": None, "time_range": {"earliest": None, "latest": None}}
    sc = np.zeros(len(seg.services), np.uint64)
    ec = np.zeros(len(seg.endpoints), np.uint64)
    out = L.SegmentSummaryC(len(seg.services), len(seg.endpoints), L.ptr(sc, C.c_uint64),
                            L.ptr(ec, C.c_uint64))
    cols = [np.ascontiguousarray(getattr(seg, k)) for k in
            ("svc", "endpoint", "is_error", "latency", "start_time")]
    ctx._check(ctx._lib.anomod_segment_summary(
        ctx.handle, L.ptr(cols[0], C.c_uint32), L.ptr(cols[1], C.c_uint32),
        L.ptr(cols[2], C.c_int32), L.ptr(cols[3], C.c_int64), L.ptr(cols[4], C.c_int64),
        seg.n, C.byref(out)))
    stats = []
    if out.latency_count:
        stats = {"min": int(out.latency_min), "max": int(out.latency_max),
                 "avg": int(out.latency_sum) / int(out.latency_count),
                 "count": int(out.latency_count)}
    tr = {"earliest": None, "latest": None}
    if out.start_count:
        tr = {"earliest": int(out.start_min), "latest": int(out.start_max)}
        tr["earliest_datetime"] = _iso_ms(tr["earliest"])
        tr["latest_datetime"] = _iso_ms(tr["latest"])
    return {
        "total_traces": int(out.total),
        "unique_services": sorted(seg.services), "unique_endpoints": sorted(seg.endpoints),
        "error_traces": int(out.error_count),
        "service_call_counts": {s: int(c) for s, c in zip(seg.services, sc)},
        "endpoint_call_counts": {e: int(c) for e, c in zip(seg.endpoints, ec)},
        "latency_stats": stats, "time_range": tr,
    }
