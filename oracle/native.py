"""ctypes binding of oracle/liboracle.so (test infrastructure only)."""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"
BINS = 896
_lib = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        _lib = C.CDLL(str(LIB))
        P = C.POINTER
        _lib.oracle_hist_bin.restype = C.c_uint32
        _lib.oracle_hist_bin.argtypes = [C.c_uint32]
        _lib.oracle_hist_bounds.argtypes = [C.c_uint32, P(C.c_uint32), P(C.c_uint32)]
        _lib.oracle_edge_aggregate.argtypes = [C.c_uint32] + [C.c_void_p] * 6 + [
            C.c_uint64, C.c_uint64] + [C.c_void_p] * 6
        _lib.oracle_quantiles.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p]
        _lib.oracle_span_edges.argtypes = [C.c_uint32] + [C.c_void_p] * 4 + [
            C.c_uint64, C.c_uint64, C.c_void_p]
        _lib.oracle_ewma_z.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_double,
                                       C.c_uint32, C.c_double, C.c_void_p]
        _lib.oracle_trace_structure.argtypes = [C.c_void_p] * 4 + [C.c_uint64, C.c_uint64,
                                                                    C.c_uint32] + [C.c_void_p] * 6
        _lib.oracle_group_by_trace.restype = C.c_int64
        _lib.oracle_group_by_trace.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p,
                                               C.c_void_p]
        _lib.oracle_take_spans.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64] + [C.c_void_p] * 12
        _lib.oracle_pagerank.restype = C.c_uint32
        _lib.oracle_pagerank.argtypes = [C.c_void_p] * 3 + [C.c_uint32, C.c_void_p, C.c_double,
                                                            C.c_uint32, C.c_double, C.c_void_p]
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def hist_bin(v: int) -> int:
    return lib().oracle_hist_bin(v)


def new_tables(S: int) -> dict:
    E = (S + 2) * S
    return {"count": np.zeros(E, np.uint64), "errors": np.zeros(E, np.uint64),
            "sum_us": np.zeros(E, np.uint64), "min_us": np.full(E, 0xFFFFFFFF, np.uint32),
            "max_us": np.zeros(E, np.uint32), "hist": np.zeros((E, BINS), np.uint64)}


def edge_aggregate(spans, S: int | None = None, t0: int = 0, t1: int | None = None,
                   tables: dict | None = None) -> dict:
    """Accumulate traces [t0, t1) of a SpanSet-like object into tables."""
    S = len(spans.services) if S is None else S
    t1 = spans.n_traces if t1 is None else t1
    tab = new_tables(S) if tables is None else tables
    arrs = [np.ascontiguousarray(getattr(spans, k)) for k in
            ("span_id", "parent_span_id", "svc", "flags", "dur_us", "trace_ptr")]
    lib().oracle_edge_aggregate(S, *[_p(a) for a in arrs], t0, t1, _p(tab["count"]),
                                _p(tab["errors"]), _p(tab["sum_us"]), _p(tab["min_us"]),
                                _p(tab["max_us"]), _p(tab["hist"]))
    return tab


def trace_structure(spans, S: int | None = None) -> dict:
    """Per-span parent_pos / depth / n_children / flags and per-trace n_roots /
    svc_mask of a SpanSet-like object (oracle_trace_structure)."""
    S = len(spans.services) if S is None else S
    words = (S + 63) // 64
    n, nt = spans.n_spans, spans.n_traces
    out = {"parent_pos": np.zeros(n, np.uint32), "depth": np.zeros(n, np.uint32),
           "n_children": np.zeros(n, np.uint32), "span_flags": np.zeros(n, np.uint8),
           "n_roots": np.zeros(nt, np.uint32), "svc_mask": np.zeros((nt, words), np.uint64)}
    arrs = [np.ascontiguousarray(getattr(spans, k)) for k in
            ("span_id", "parent_span_id", "svc", "trace_ptr")]
    lib().oracle_trace_structure(*[_p(a) for a in arrs], 0, nt, words,
                                 *[_p(out[k]) for k in ("parent_pos", "depth", "n_children",
                                                        "span_flags", "n_roots", "svc_mask")])
    return out


def span_edges(spans, S: int | None = None) -> np.ndarray:
    """Edge row of every span (first-match parent rule of the aggregation)."""
    S = len(spans.services) if S is None else S
    arrs = [np.ascontiguousarray(getattr(spans, k)) for k in
            ("span_id", "parent_span_id", "svc", "trace_ptr")]
    out = np.zeros(spans.n_spans, np.uint32)
    lib().oracle_span_edges(S, *[_p(a) for a in arrs], 0, spans.n_traces, _p(out))
    return out


def exact_quantiles(spans, q_pct=(50, 99), S: int | None = None) -> np.ndarray:
    """Per edge: sorted(latencies)[int(c * (q / 100))] (monitor_http_responses.py:
    180-190 nearest rank, the f64 product truncated as Python's int() does),
    NaN for an empty edge; [E, len(q)]."""
    S = len(spans.services) if S is None else S
    E = (S + 2) * S
    e = span_edges(spans, S)
    order = np.lexsort((spans.dur_us, e))
    es, ds = e[order], spans.dur_us[order]
    cnt = np.bincount(es, minlength=E)
    start = np.r_[0, np.cumsum(cnt)[:-1]]
    out = np.full((E, len(q_pct)), np.nan)
    for k, q in enumerate(q_pct):
        nz = cnt > 0
        rank = (cnt[nz].astype(np.float64) * (q / 100)).astype(np.int64)
        out[nz, k] = ds[start[nz] + rank]
    return out


def quantiles(hist: np.ndarray, q_pct: int) -> np.ndarray:
    hist = np.ascontiguousarray(hist, np.uint64)
    out = np.empty(hist.shape[0])
    lib().oracle_quantiles(_p(hist), hist.shape[0], q_pct, _p(out))
    return out


def finalize(tab: dict) -> dict:
    tab["p50_us"] = quantiles(tab["hist"], 50)
    tab["p99_us"] = quantiles(tab["hist"], 99)
    return tab


def ewma_z(X: np.ndarray, alpha: float, W: int, eps: float = 1e-12) -> np.ndarray:
    X = np.ascontiguousarray(X, np.float32)
    T, S = X.shape
    Z = np.empty((T // W, S), np.float32)
    lib().oracle_ewma_z(_p(X), T, S, alpha, W, eps, _p(Z))
    return Z


def pagerank(row_ptr, col, w, p, alpha=0.85, iters=100, tol=1e-10):
    row_ptr = np.ascontiguousarray(row_ptr, np.uint32)
    col = np.ascontiguousarray(col, np.uint32)
    w = np.ascontiguousarray(w, np.float32)
    p = np.asarray(p, np.float64)
    p = np.ascontiguousarray(p / p.sum())
    N = row_ptr.shape[0] - 1
    x = np.empty(N)
    if col.size == 0:
        col, w = np.zeros(1, np.uint32), np.zeros(1, np.float32)
    it = lib().oracle_pagerank(_p(row_ptr), _p(col), _p(w), N, _p(p), alpha, iters, tol, _p(x))
    return x, it


def group_by_trace(trace_hash: np.ndarray, threads: int = 1) -> tuple[np.ndarray, np.ndarray]:
    """(order, trace_ptr) of oracle_group_by_trace: spans taken in `order` are
    grouped (traces by mix64(trace_hash) ascending, spans of a trace in
    arrival order) — spec.group_by_trace as a parallel C radix partition."""
    h = np.ascontiguousarray(trace_hash, np.uint64)
    n = h.shape[0]
    order = np.empty(n, np.uint64)
    tptr = np.empty(n + 1, np.uint64)
    nt = lib().oracle_group_by_trace(_p(h), n, threads, _p(order), _p(tptr))
    if nt < 0:
        raise MemoryError("oracle_group_by_trace failed")
    return order.astype(np.int64), tptr[:nt + 1].copy()

