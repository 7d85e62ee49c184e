"""API-response summaries (second half): the drop-ins
for the SocialNetwork OpenAPI monitors' report writers.

* ``generate_summary`` — OpenAPIResponseCollector.generate_summary
  (SN_collection-scripts/Dataset/api_responses/monitor_http_responses.py:
  150-207): status-code / content-type distributions, error count, success
  rate and the latency statistics of ``latency_ms > 0``.
* ``generate_reports`` — EnhancedOpenAPIMonitor.generate_reports
  (enhanced_openapi_monitor.py:318-393): response_summary.json,
  status_code_distribution.csv and endpoint_performance.json.

The latency statistics (select, sort, nearest-rank picks, min / max / sum)
and the distributions run in libanomod (``anomod_response_summary`` /
``anomod_value_summary``, csrc/summary.hip); turning response dicts into
columns and the JSON / CSV formatting are host work restated from the
reference.  Order statistics are exact; ``mean`` is the device sum over the
sorted values / count — equal to the reference whenever the sum is exact
(integer latencies), else within count * 2^-53 relative.
"""
from __future__ import annotations

import ctypes as C
import json
from datetime import datetime
from pathlib import Path

import numpy as np

from . import _lib as L

_PICKS = ("min", "max", "mean", "median", "p95", "p99")


def _context(ctx):
    if ctx is not None:
        return ctx
    from .engine import default_context
    return default_context()


def _python_value(v: float, rank: int, values: list, sorted_arr: np.ndarray):
    """The Python object ``sorted(values)[rank]`` is, given that its value is
    ``v``: int latencies stay int in the reference's JSON.  Mixed int / float
    inputs resolve ties the way the stable sort does (original order among
    equal values)."""
    kinds = {type(x) for x in values}
    if kinds <= {int}:
        return int(v)
    if kinds <= {float}:
        return float(v)
    first = int(np.searchsorted(sorted_arr, v, side="left"))
    equal = [x for x in values if x == v]
    return equal[rank - first]


def _stats_dict(s: L.ValueSummaryC, values: list, sorted_pos: np.ndarray | None,
                suffix: str) -> dict:
    if s.count == 0:
        return {}
    c = int(s.count)
    ranks = {"min": 0, "max": c - 1, "median": c // 2, "p95": int(c * 0.95),
             "p99": int(c * 0.99)}
    out = {}
    for k in _PICKS:
        if k == "mean":
            total = s.sum
            if all(type(x) is int for x in values):
                total = int(total)  # exact below 2^53: the reference's int sum
            out["mean" + suffix] = total / c
            continue
        out[k + suffix] = _python_value(getattr(s, k), ranks[k], values, sorted_pos)
    return out


def value_statistics(ctx, values, *, positive_only: bool = True, suffix: str = "") -> dict:
    """min / max / mean / median / p95 / p99 of ``values`` (generate_summary's
    ``latency_statistics`` with positive_only, generate_reports' with
    ``positive_only=False, suffix='_ms'``); {} when nothing is selected."""
    ctx = _context(ctx)
    vals = list(values)
    arr = np.ascontiguousarray(np.asarray(vals, dtype=np.float64).reshape(-1))
    if not positive_only and np.isnan(arr).any():
        raise ValueError("NaN latency: the reference's sorted() has no defined order")
    out = L.ValueSummaryC()
    ctx._check(ctx._lib.anomod_value_summary(ctx.handle, L.ptr(arr, C.c_double), arr.size,
                                             1 if positive_only else 0, C.byref(out)))
    sel = [x for x in vals if x > 0] if positive_only else vals
    mixed = len({type(x) for x in sel}) > 1
    return _stats_dict(out, sel, np.sort(np.asarray(sel, np.float64)) if mixed else None, suffix)


def _first_appearance_ids(keys: list) -> tuple[np.ndarray, list]:
    index: dict = {}
    ids = np.fromiter((index.setdefault(k, len(index)) for k in keys), np.uint32, len(keys))
    return ids, list(index)


def summarize_responses(ctx, responses: list[dict], *, start_time: float, duration,
                        endpoints) -> dict | None:
    """The dict generate_summary writes (None for no responses: the reference
    returns before writing, :152-153)."""
    if not responses:
        return None
    ctx = _context(ctx)
    n = len(responses)
    status_ids, statuses = _first_appearance_ids([r.get("status_code", 0) for r in responses])
    ctype_ids, ctypes_ = _first_appearance_ids(
        [r.get("content_type", "unknown").split(";")[0] for r in responses])
    has_error = np.fromiter(("error" in r for r in responses), np.uint8, n)
    lat_py = [r.get("latency_ms", 0) for r in responses]
    lat = np.asarray(lat_py, np.float64)
    sc = np.zeros(len(statuses), np.uint64)
    cc = np.zeros(len(ctypes_), np.uint64)
    out = L.ResponseSummaryC(len(statuses), len(ctypes_), L.ptr(sc, C.c_uint64),
                             L.ptr(cc, C.c_uint64))
    ctx._check(ctx._lib.anomod_response_summary(
        ctx.handle, L.ptr(status_ids, C.c_uint32), L.ptr(ctype_ids, C.c_uint32),
        L.ptr(has_error, C.c_uint8), L.ptr(lat, C.c_double), n, C.byref(out)))
    sel = [x for x in lat_py if x > 0]
    mixed = len({type(x) for x in sel}) > 1
    errors = int(out.error_count)
    return {
        "collection_info": {
            "start_time": datetime.fromtimestamp(start_time).isoformat(),
            "duration_seconds": duration,
            "total_responses": n,
            "endpoints_monitored": endpoints,
        },
        "status_code_distribution": {s: int(c) for s, c in zip(statuses, sc)},
        "latency_statistics": _stats_dict(out.latency, sel,
                                          np.sort(np.asarray(sel, np.float64)) if mixed
                                          else None, ""),
        "content_type_distribution": {t: int(c) for t, c in zip(ctypes_, cc)},
        "error_count": errors,
        "success_rate": (n - errors) / n * 100,
    }


def generate_summary(ctx, responses: list[dict], summary_file, *, start_time: float, duration,
                     endpoints) -> bool:
    """Write generate_summary's JSON (indent=2); False (nothing written) for
    no responses."""
    summary = summarize_responses(ctx, responses, start_time=start_time, duration=duration,
                                  endpoints=endpoints)
    if summary is None:
        return False
    with open(summary_file, "w") as f:
        json.dump(summary, f, indent=2)
    return True


def response_reports(ctx, responses: list[dict], stats: dict, *, start_time: float, duration,
                     endpoints, sample_interval) -> tuple[dict, str, dict]:
    """(response_summary dict, status_code_distribution.csv text,
    endpoint_performance dict) of generate_reports (:318-393).  ``stats`` is
    the monitor's running counters (total/successful/failed_requests,
    status_codes, response_times, errors; :71-76)."""
    times = list(stats.get("response_times", []))
    latency = value_statistics(ctx, times, positive_only=False, suffix="_ms") if times else {}
    codes = dict(stats.get("status_codes", {}))
    errs = list(stats.get("errors", []))
    total_req = stats.get("total_requests", 0)
    ok_req = stats.get("successful_requests", 0)
    summary = {
        "collection_info": {
            "start_time": datetime.fromtimestamp(start_time).isoformat(),
            "duration_seconds": duration,
            "total_responses": len(responses),
            "endpoints_monitored": endpoints,
            "sample_interval_seconds": sample_interval,
        },
        "statistics": {
            "total_requests": total_req,
            "successful_requests": ok_req,
            "failed_requests": stats.get("failed_requests", 0),
            "success_rate_percent": (ok_req / max(1, total_req)) * 100,
        },
        "status_code_distribution": codes,
        "latency_statistics": latency,
        "error_summary": {
            "total_errors": len(errs),
            "unique_errors": len(set(errs)),
            "common_errors": list(set(errs)),  # set order, as the reference (:353)
        },
    }
    lines = ["status_code,count,percentage\n"]
    total = sum(codes.values())
    for code, count in sorted(codes.items()):
        pct = (count / total * 100) if total > 0 else 0
        lines.append(f"{code},{count},{pct:.2f}\n")
    # per endpoint, first-appearance order: count, mean latency (a left-to-right
    # sum per endpoint, as np.bincount accumulates), status-code counts
    ep_ids, eps = _first_appearance_ids([r.get("endpoint", "unknown") for r in responses])
    lat = np.asarray([r.get("latency_ms", 0) for r in responses], np.float64)
    counts = np.bincount(ep_ids, minlength=len(eps)) if len(eps) else np.zeros(0, np.int64)
    sums = np.bincount(ep_ids, weights=lat, minlength=len(eps)) if len(eps) else counts
    per_status: list[dict] = [dict() for _ in eps]
    for e, r in zip(ep_ids, responses):
        st = r.get("status_code", 0)
        per_status[e][st] = per_status[e].get(st, 0) + 1
    perf = {ep: {"count": int(counts[i]), "avg_latency": float(sums[i]) / int(counts[i]),
                 "status_codes": per_status[i]} for i, ep in enumerate(eps)}
    return summary, "".join(lines), perf


def generate_reports(ctx, responses: list[dict], stats: dict, output_dir, *, start_time: float,
                     duration, endpoints, sample_interval) -> None:
    """Write the three report files generate_reports writes into output_dir."""
    out = Path(output_dir)
    summary, csv_text, perf = response_reports(
        ctx, responses, stats, start_time=start_time, duration=duration, endpoints=endpoints,
        sample_interval=sample_interval)
    with open(out / "response_summary.json", "w") as f:
        json.dump(summary, f, indent=2)
    with open(out / "status_code_distribution.csv", "w") as f:
        f.write(csv_text)
    with open(out / "endpoint_performance.json", "w") as f:
        json.dump(perf, f, indent=2)
