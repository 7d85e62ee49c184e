"""Host containers: span sets (struct-of-arrays) and edge tables.

A :class:`SpanSet` is the columnar form of the spans the reference collectors
write one dict (or CSV row) at a time — jaeger_to_csv.py:76-90 for SN,
trace_collector.py:86-123 (SpanRecord.to_dict) for TT.  Spans are grouped by
trace: trace t owns rows [trace_ptr[t], trace_ptr[t+1]).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib as L


@dataclass
class SpanSet:
    services: list[str]
    trace_ptr: np.ndarray      # u64 [n_traces + 1]
    trace_hash: np.ndarray     # u64 [n_spans]
    span_id: np.ndarray        # u64 [n_spans]
    parent_span_id: np.ndarray  # u64 [n_spans]; 0 = no parent reference
    svc: np.ndarray            # u16 [n_spans]
    flags: np.ndarray          # u16 [n_spans]
    dur_us: np.ndarray         # u32 [n_spans]
    trace_ids: list[str] | None = None
    # span ids unique within every trace (the producer's declaration, or
    # check_unique_ids()): lets the GPU parent lookups scan from both ends
    unique_ids: bool = False
    # performance hints the library learns on the device at a set's first
    # aggregation (include/anomod.h anomod_spans_hints): parent-scan order
    # (1 collector order / 0 shuffled / -1 unknown) and histogram form (0 pair
    # / 1 compact / -1 unknown).  Context.upload hands them to every upload
    # and edge_aggregate keeps what was learned, so a host set that is
    # uploaded per call (features()) learns them once.  Results never depend
    # on them.
    scan_order: int = field(default=-1, compare=False)
    hist_form: int = field(default=-1, compare=False)
    _keep: list = field(default_factory=list, repr=False, compare=False)

    def __post_init__(self):
        self.trace_ptr = np.ascontiguousarray(self.trace_ptr, dtype=np.uint64)
        self.trace_hash = np.ascontiguousarray(self.trace_hash, dtype=np.uint64)
        self.span_id = np.ascontiguousarray(self.span_id, dtype=np.uint64)
        self.parent_span_id = np.ascontiguousarray(self.parent_span_id, dtype=np.uint64)
        self.svc = np.ascontiguousarray(self.svc, dtype=np.uint16)
        self.flags = np.ascontiguousarray(self.flags, dtype=np.uint16)
        self.dur_us = np.ascontiguousarray(self.dur_us, dtype=np.uint32)
        n = self.span_id.shape[0]
        for name in ("trace_hash", "parent_span_id", "svc", "flags", "dur_us"):
            if getattr(self, name).shape[0] != n:
                raise ValueError(f"SpanSet column {name} has {getattr(self, name).shape[0]} rows, "
                                 f"expected {n}")
        if self.trace_ptr.shape[0] < 1:
            raise ValueError("trace_ptr needs at least one entry")

    @property
    def n_spans(self) -> int:
        return int(self.span_id.shape[0])

    @property
    def n_traces(self) -> int:
        return int(self.trace_ptr.shape[0] - 1)

    @property
    def n_services(self) -> int:
        return len(self.services)

    def soa(self) -> L.SpanSoA:
        return L.SpanSoA(
            L.ptr(self.trace_hash, C.c_uint64), L.ptr(self.span_id, C.c_uint64),
            L.ptr(self.parent_span_id, C.c_uint64), L.ptr(self.svc, C.c_uint16),
            L.ptr(self.flags, C.c_uint16), L.ptr(self.dur_us, C.c_uint32))

    def check_unique_ids(self) -> bool:
        """Exact: no trace holds a span id twice (sets and returns
        unique_ids)."""
        if self.n_spans:
            t = self.trace_of_span()
            order = np.lexsort((self.span_id, t))
            ts, ids = t[order], self.span_id[order]
            self.unique_ids = not bool(np.any((ts[1:] == ts[:-1]) & (ids[1:] == ids[:-1])))
        else:
            self.unique_ids = True
        return self.unique_ids

    def trace_of_span(self) -> np.ndarray:
        """Trace index of every span (host helper)."""
        lens = np.diff(self.trace_ptr).astype(np.int64)
        return np.repeat(np.arange(self.n_traces, dtype=np.int64), lens)

    def select_traces(self, mask: np.ndarray) -> "SpanSet":
        """Sub-set of whole traces (trace order preserved)."""
        mask = np.asarray(mask, dtype=bool)
        lens = np.diff(self.trace_ptr).astype(np.int64)
        span_mask = np.repeat(mask, lens)
        new_ptr = np.zeros(int(mask.sum()) + 1, dtype=np.uint64)
        np.cumsum(lens[mask], out=new_ptr[1:])
        ids = None
        if self.trace_ids is not None:
            ids = [t for t, m in zip(self.trace_ids, mask) if m]
        return SpanSet(list(self.services), new_ptr, self.trace_hash[span_mask],
                       self.span_id[span_mask], self.parent_span_id[span_mask],
                       self.svc[span_mask], self.flags[span_mask], self.dur_us[span_mask], ids,
                       self.unique_ids)

    def shard(self, nshards: int, rank: int) -> "SpanSet":
        """Traces whose trace_hash % nshards == rank."""
        if self.n_traces == 0:
            return self.select_traces(np.zeros(0, dtype=bool))
        first = self.trace_ptr[:-1].astype(np.int64)
        lens = np.diff(self.trace_ptr).astype(np.int64)
        h = np.zeros(self.n_traces, dtype=np.uint64)
        nz = lens > 0
        h[nz] = self.trace_hash[first[nz]]
        return self.select_traces((h % np.uint64(nshards)) == np.uint64(rank))

    def observed_services(self) -> "SpanSet":
        """The same spans over only the services they name (names stay sorted,
        ids renumbered) — what a collector payload records as
        metadata.services_discovered = sorted(union of observed services),
        trace_collector.py:572."""
        used = np.unique(self.svc)
        if used.shape[0] == len(self.services):
            return self
        remap = np.zeros(len(self.services), np.uint16)
        remap[used] = np.arange(used.shape[0], dtype=np.uint16)
        return SpanSet([self.services[i] for i in used.tolist()], self.trace_ptr, self.trace_hash,
                       self.span_id, self.parent_span_id, remap[self.svc], self.flags,
                       self.dur_us, self.trace_ids, self.unique_ids)

    def take(self, order: np.ndarray, trace_ptr: np.ndarray) -> "SpanSet":
        """The spans in `order`, split into traces by `trace_ptr`."""
        return SpanSet(self.services, trace_ptr, self.trace_hash[order], self.span_id[order],
                       self.parent_span_id[order], self.svc[order], self.flags[order],
                       self.dur_us[order])

    @staticmethod
    def concat(sets: list["SpanSet"]) -> "SpanSet":
        if not sets:
            raise ValueError("concat of no span sets")
        services = sets[0].services
        for s in sets[1:]:
            if s.services != services:
                raise ValueError("span sets with different service lists")
        lens = np.concatenate([np.diff(s.trace_ptr) for s in sets]).astype(np.uint64)
        ptr = np.zeros(lens.shape[0] + 1, dtype=np.uint64)
        np.cumsum(lens, out=ptr[1:])
        cat = lambda name: np.concatenate([getattr(s, name) for s in sets])  # noqa: E731
        ids = None
        if all(s.trace_ids is not None for s in sets):
            ids = [t for s in sets for t in s.trace_ids]
        return SpanSet(list(services), ptr, cat("trace_hash"), cat("span_id"),
                       cat("parent_span_id"), cat("svc"), cat("flags"), cat("dur_us"), ids,
                       all(s.unique_ids for s in sets))


def edge_rows(n_services: int) -> int:
    return (n_services + L.ROOT_ROWS) * n_services


@dataclass
class EdgeTable:
    """Per (parent service -> child service) edge aggregate.

    Row r = p * S + c; p == S is ROOT (no parent reference), p == S + 1 is
    ORPHAN (parent reference not found in the trace)."""

    services: list[str]
    count: np.ndarray    # u64 [E]
    errors: np.ndarray   # u64 [E]
    sum_us: np.ndarray   # u64 [E]
    min_us: np.ndarray   # u32 [E]
    max_us: np.ndarray   # u32 [E]
    p50_us: np.ndarray   # f64 [E]
    p99_us: np.ndarray   # f64 [E]
    hist: np.ndarray | None = None  # u64 [E, HIST_BINS]

    @property
    def n_services(self) -> int:
        return len(self.services)

    @staticmethod
    def empty(services: list[str], with_hist: bool = True) -> "EdgeTable":
        E = edge_rows(len(services))
        return EdgeTable(list(services), np.zeros(E, np.uint64), np.zeros(E, np.uint64),
                         np.zeros(E, np.uint64), np.full(E, 0xFFFFFFFF, np.uint32),
                         np.zeros(E, np.uint32), np.full(E, np.nan), np.full(E, np.nan),
                         np.zeros((E, L.HIST_BINS), np.uint64) if with_hist else None)

    def c_struct(self) -> L.EdgeTableC:
        return L.EdgeTableC(
            self.n_services, L.HIST_BINS, L.ptr(self.count, C.c_uint64),
            L.ptr(self.errors, C.c_uint64), L.ptr(self.sum_us, C.c_uint64),
            L.ptr(self.min_us, C.c_uint32), L.ptr(self.max_us, C.c_uint32),
            L.ptr(self.hist, C.c_uint64), L.ptr(self.p50_us, C.c_double),
            L.ptr(self.p99_us, C.c_double))

    def parent_name(self, p: int) -> str:
        S = self.n_services
        return "ROOT" if p == S else "ORPHAN" if p == S + 1 else self.services[p]

    def records(self) -> list[dict]:
        """Non-empty edges as dicts (parent, child, count, errors, mean/p50/p99)."""
        S = self.n_services
        out = []
        for r in np.nonzero(self.count)[0]:
            p, c = divmod(int(r), S)
            n = int(self.count[r])
            out.append({
                "parent": self.parent_name(p), "child": self.services[c], "count": n,
                "errors": int(self.errors[r]), "mean_us": int(self.sum_us[r]) / n,
                "min_us": int(self.min_us[r]), "max_us": int(self.max_us[r]),
                "p50_us": float(self.p50_us[r]), "p99_us": float(self.p99_us[r]),
            })
        return out

    def call_graph(self) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Cross-service caller -> callee CSR (self edges, ROOT, ORPHAN dropped);
        weight = call count."""
        S = self.n_services
        cnt = self.count[: S * S].reshape(S, S).astype(np.float64)
        np.fill_diagonal(cnt, 0.0)
        row_ptr = np.zeros(S + 1, dtype=np.uint32)
        cols, ws = [], []
        for p in range(S):
            nz = np.nonzero(cnt[p])[0]
            cols.extend(nz.tolist())
            ws.extend(cnt[p, nz].tolist())
            row_ptr[p + 1] = len(cols)
        return row_ptr, np.asarray(cols, dtype=np.uint32), np.asarray(ws, dtype=np.float32)


@dataclass
class TraceStructure:
    """Per-span / per-trace structure of a span set (trace_collector.py:401-481,
    536-547; see anomod_trace_structure in include/anomod.h)."""

    services: list[str]
    parent_pos: np.ndarray   # u32 [n_spans] position of the node's parent in its trace
    depth: np.ndarray        # u32 [n_spans]
    n_children: np.ndarray   # u32 [n_spans]
    span_flags: np.ndarray   # u8  [n_spans] SPAN_ROOT | SPAN_FIRST
    n_roots: np.ndarray      # u32 [n_traces]
    svc_mask: np.ndarray     # u64 [n_traces, ceil(S/64)]

    @staticmethod
    def empty(services: list[str], n_spans: int, n_traces: int) -> "TraceStructure":
        w = (len(services) + 63) // 64
        return TraceStructure(list(services), np.zeros(n_spans, np.uint32),
                              np.zeros(n_spans, np.uint32), np.zeros(n_spans, np.uint32),
                              np.zeros(n_spans, np.uint8), np.zeros(n_traces, np.uint32),
                              np.zeros((n_traces, w), np.uint64))

    def c_struct(self) -> L.TraceStructC:
        return L.TraceStructC(len(self.services), L.ptr(self.parent_pos, C.c_uint32),
                              L.ptr(self.depth, C.c_uint32), L.ptr(self.n_children, C.c_uint32),
                              L.ptr(self.span_flags, C.c_uint8), L.ptr(self.n_roots, C.c_uint32),
                              L.ptr(self.svc_mask, C.c_uint64))

    def services_involved(self, t: int) -> list[str]:
        """Sorted service names of trace t (trace_collector.py:536)."""
        m = self.svc_mask[t]
        return [s for i, s in enumerate(self.services) if (int(m[i // 64]) >> (i % 64)) & 1]

    def root_positions(self, trace_ptr: np.ndarray, t: int) -> list[int]:
        """Trace-local positions of the root nodes of trace t, in first-seen
        order (root_span_node_ids, trace_collector.py:443, 544)."""
        a, b = int(trace_ptr[t]), int(trace_ptr[t + 1])
        fl = self.span_flags[a:b]
        return [k for k in range(b - a) if fl[k] == (L.SPAN_ROOT | L.SPAN_FIRST)]
