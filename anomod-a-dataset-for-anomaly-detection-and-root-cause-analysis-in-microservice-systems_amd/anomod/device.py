"""Device context: one HIP device + stream (+ optional RCCL communicator).

Thin object layer over the C ABI; every compute method runs a hand-written
HIP kernel in libanomod.so.  Nothing here falls back to the CPU.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib as L
from .spans import EdgeTable, SpanSet, TraceStructure, edge_rows


@dataclass
class SynthSpec:
    """Synthetic workload: topology 'SN' or 'TT' (or 'LONG':
    SN services in traces of 16..4000 spans, the length / depth stress case)."""

    topology: str = "SN"
    seed: int = 20251103
    fault_service: str | int | None = None
    fault_latency_mult: int = 8
    p_error_ppm: int = 5000          # 0.5 % base error rate
    p_fault_error_ppm: int = 200000  # 20 % on the faulty service
    p_orphan_ppm: int = 0

    @property
    def topo_id(self) -> int:
        return {"SN": L.TOPO_SN, "TT": L.TOPO_TT, "LONG": L.TOPO_LONG}[self.topology.upper()]

    def services(self) -> list[str]:
        return synth_services(self.topology)

    def c_struct(self) -> L.SynthSpec:
        fault = 0xFFFFFFFF
        if self.fault_service is not None:
            fault = (self.services().index(self.fault_service)
                     if isinstance(self.fault_service, str) else int(self.fault_service))
        return L.SynthSpec(self.topo_id, fault, self.seed, self.fault_latency_mult,
                           self.p_error_ppm, self.p_fault_error_ppm, self.p_orphan_ppm)


def synth_services(topology: str) -> list[str]:
    lib = L.lib()
    tid = {"SN": L.TOPO_SN, "TT": L.TOPO_TT, "LONG": L.TOPO_LONG}[topology.upper()]
    n = C.c_uint32()
    L.check(lib.anomod_synth_n_services(tid, C.byref(n)))
    return [lib.anomod_synth_service_name(tid, i).decode() for i in range(n.value)]


def synth_generate_host(spec: SynthSpec, n_traces: int, shard: int = 0) -> SpanSet:
    """Generate a synthetic span set on the host (same generator as the GPU)."""
    lib = L.lib()
    cs = spec.c_struct()
    n = C.c_uint64()
    L.check(lib.anomod_synth_count_host(C.byref(cs), shard, n_traces, C.byref(n)))
    ns = n.value
    arr = dict(trace_hash=np.empty(ns, np.uint64), span_id=np.empty(ns, np.uint64),
               parent_span_id=np.empty(ns, np.uint64), svc=np.empty(ns, np.uint16),
               flags=np.empty(ns, np.uint16), dur_us=np.empty(ns, np.uint32))
    ptr = np.empty(n_traces + 1, np.uint64)
    L.check(lib.anomod_synth_generate_host(C.byref(cs), shard, n_traces,
                                           C.byref(_soa_out(arr)), L.ptr(ptr, C.c_uint64)))
    # span ids are injective in the span index (csrc/synth.h synth_span_id)
    return SpanSet(spec.services(), ptr, **arr, unique_ids=True, scan_order=1)


def _soa_out(arr: dict) -> L.SpanSoA:
    return L.SpanSoA(L.ptr(arr["trace_hash"], C.c_uint64), L.ptr(arr["span_id"], C.c_uint64),
                     L.ptr(arr["parent_span_id"], C.c_uint64), L.ptr(arr["svc"], C.c_uint16),
                     L.ptr(arr["flags"], C.c_uint16), L.ptr(arr["dur_us"], C.c_uint32))


def device_count() -> int:
    n = C.c_int()
    L.check(L.lib().anomod_device_count(C.byref(n)))
    return n.value


def device_count_safe() -> int:
    """Number of visible GPUs, 0 when the HIP runtime reports none."""
    n = C.c_int()
    return n.value if L.lib().anomod_device_count(C.byref(n)) == L.OK else 0


class DeviceSpans:
    """A span set resident in HBM (owned by libanomod)."""

    def __init__(self, ctx: "Context", handle: C.c_void_p, services: list[str]):
        self.ctx, self.handle, self.services = ctx, handle, list(services)
        ns, nt, g = C.c_uint64(), C.c_uint64(), C.c_int()
        L.check(L.lib().anomod_spans_info(handle, C.byref(ns), C.byref(nt)))
        L.check(L.lib().anomod_spans_grouped(handle, C.byref(g)))
        self.n_spans, self.n_traces = ns.value, nt.value
        self.grouped = bool(g.value)  # False: arrival order, traces known by trace_hash only

    @property
    def unique_ids(self) -> bool:
        u = C.c_int()
        L.check(L.lib().anomod_spans_unique_ids(self.handle, C.byref(u)))
        return bool(u.value)

    @property
    def scan_order(self) -> int:
        """1 collector order / 0 shuffled inside traces / -1 not probed yet."""
        o = C.c_int()
        L.check(L.lib().anomod_spans_scan_order(self.handle, C.byref(o)))
        return o.value

    @property
    def hist_compact(self) -> bool:
        """True once an aggregation overflowed the pair-form LDS histogram
        (later ones use the compact form)."""
        c = C.c_int()
        L.check(L.lib().anomod_spans_hist_compact(self.handle, C.byref(c)))
        return bool(c.value)

    @unique_ids.setter
    def unique_ids(self, v: bool):
        L.check(L.lib().anomod_spans_set_unique_ids(self.handle, 1 if v else 0))

    @property
    def hints(self) -> tuple[int, int]:
        """(scan_order, hist_form) the library holds for this set."""
        o, f = C.c_int(), C.c_int()
        L.check(L.lib().anomod_spans_hints(self.handle, C.byref(o), C.byref(f)))
        return o.value, f.value

    def set_hints(self, scan_order: int, hist_form: int):
        L.check(L.lib().anomod_spans_set_hints(self.handle, scan_order, hist_form))

    def download(self) -> SpanSet:
        n = self.n_spans
        arr = dict(trace_hash=np.empty(n, np.uint64), span_id=np.empty(n, np.uint64),
                   parent_span_id=np.empty(n, np.uint64), svc=np.empty(n, np.uint16),
                   flags=np.empty(n, np.uint16), dur_us=np.empty(n, np.uint32))
        ptr = np.empty(self.n_traces + 1, np.uint64)
        L.check(L.lib().anomod_spans_download(self.ctx.handle, self.handle,
                                              C.byref(_soa_out(arr)), L.ptr(ptr, C.c_uint64)),
                self.ctx.handle)
        order, form = self.hints
        return SpanSet(self.services, ptr, **arr, unique_ids=self.unique_ids, scan_order=order,
                       hist_form=form)

    def free(self):
        if self.handle:
            L.lib().anomod_spans_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Context:
    """One GPU: ``Context(device)``; use as a context manager or call close()."""

    def __init__(self, device: int = 0):
        self._lib = L.lib()
        h = C.c_void_p()
        L.check(self._lib.anomod_ctx_create(device, C.byref(h)))
        self.handle = h
        self.device = device

    # -- lifecycle
    def close(self):
        if self.handle:
            self._lib.anomod_ctx_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, status: int):
        L.check(status, self.handle)

    def synchronize(self):
        self._check(self._lib.anomod_ctx_synchronize(self.handle))

    def stage_ms(self, stage: int) -> float:
        v = C.c_double()
        self._check(self._lib.anomod_ctx_stage_ms(self.handle, stage, C.byref(v)))
        return v.value

    def host_ms(self) -> dict:
        """Host wall milliseconds of the last occurrence of each one-off setup
        step / host-side call phase (anomod_ctx_host_ms) and how many times it
        happened: {name: (ms, count)}."""
        out = {}
        for slot, name in enumerate(L.HOST_SLOT_NAMES):
            v, c = C.c_double(), C.c_uint64()
            self._check(self._lib.anomod_ctx_host_ms(self.handle, slot, C.byref(v), C.byref(c)))
            out[name] = (v.value, c.value)
        return out

    def group_info(self) -> dict:
        """How the last grouping ran: path ("bucket" / "join": the bucket
        scatters then the ungrouped aggregation's per-bucket hash join /
        "fused-sort": the same scatters then the sorting bucket kernels' edge
        records (ANOMOD_FUSED_JOIN=0) / "lsd"),
        scatter levels or radix passes, and the key bits they sorted on."""
        p, lv, b = C.c_int(), C.c_int(), C.c_int()
        self._check(self._lib.anomod_ctx_group_info(self.handle, C.byref(p), C.byref(lv),
                                                    C.byref(b)))
        return {"path": {1: "bucket", 2: "join", 3: "fused-sort"}.get(p.value, "lsd"), "levels": lv.value,
                "bits": b.value}

    # -- multi-GPU
    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * L.UNIQUE_ID_BYTES)()
        L.check(L.lib().anomod_comm_unique_id(buf))
        return bytes(buf)

    def attach_comm(self, unique_id: bytes, nranks: int, rank: int):
        buf = (C.c_uint8 * L.UNIQUE_ID_BYTES).from_buffer_copy(unique_id)
        self._check(self._lib.anomod_ctx_attach_comm(self.handle, buf, nranks, rank))

    def comm_info(self) -> tuple[int, int]:
        """(nranks, rank) of the attached transport ((1, 0) without one)."""
        n, r = C.c_int(), C.c_int()
        self._check(self._lib.anomod_ctx_comm_info(self.handle, C.byref(n), C.byref(r)))
        return n.value, r.value

    def sort_u64(self, keys, begin_bit: int = 0, end_bit: int = 64) -> tuple[np.ndarray, int]:
        """Stable device radix sort of u64 keys by bits [begin_bit, end_bit)
        (csrc/radix.hip) -> (sorted keys, digit passes run)."""
        k = np.ascontiguousarray(keys, np.uint64)
        out = np.empty_like(k)
        passes = C.c_int()
        self._check(self._lib.anomod_sort_u64(self.handle, L.ptr(k, C.c_uint64), k.size,
                                              begin_bit, end_bit, L.ptr(out, C.c_uint64),
                                              C.byref(passes)))
        return out, passes.value

    def attach_host_comm(self, nranks: int, rank: int, allreduce, allgather):
        """Host collective transport instead of RCCL: ``allreduce(buf, dtype,
        op)`` reduces a numpy array in place over all ranks, ``allgather(buf,
        block)`` fills every rank's ``block``-byte slice of a u8 array (this
        rank's is set); libanomod stages every collective through pinned host
        memory and calls them in the RCCL path's order."""
        dtypes = {L.DTYPE_I32: np.int32, L.DTYPE_U32: np.uint32, L.DTYPE_U64: np.uint64,
                  L.DTYPE_F64: np.float64}

        def _ar(_user, buf, count, dtype, op):
            try:
                dt = np.dtype(dtypes[dtype])
                raw = (C.c_uint8 * (count * dt.itemsize)).from_address(buf)
                allreduce(np.frombuffer(raw, dtype=dt), dtype, op)
                return 0
            except Exception:  # noqa: BLE001 - reported to libanomod as a failed transport
                return 1

        def _ag(_user, buf, block):
            try:
                raw = (C.c_uint8 * (block * nranks)).from_address(buf)
                allgather(np.frombuffer(raw, dtype=np.uint8), block)
                return 0
            except Exception:  # noqa: BLE001
                return 1

        # the ctypes thunks must outlive every call libanomod makes through them
        self._host_comm = (L.HostAllreduceFn(_ar), L.HostAllgatherFn(_ag))
        self._check(self._lib.anomod_ctx_attach_host_comm(
            self.handle, nranks, rank, C.cast(self._host_comm[0], C.c_void_p),
            C.cast(self._host_comm[1], C.c_void_p), None))

    # -- spans
    def upload(self, spans: SpanSet) -> DeviceSpans:
        h = C.c_void_p()
        soa = spans.soa()
        self._check(self._lib.anomod_spans_upload(self.handle, C.byref(soa), spans.n_spans,
                                                  L.ptr(spans.trace_ptr, C.c_uint64),
                                                  spans.n_traces, C.byref(h)))
        d = DeviceSpans(self, h, spans.services)
        d.unique_ids = spans.unique_ids
        d.set_hints(spans.scan_order, spans.hist_form)
        return d

    def upload_ungrouped(self, spans: SpanSet) -> DeviceSpans:
        """Upload spans in arrival order: the trace of a span is its trace_hash
        alone (spans.trace_ptr is ignored)."""
        h = C.c_void_p()
        soa = spans.soa()
        self._check(self._lib.anomod_spans_upload_ungrouped(self.handle, C.byref(soa),
                                                            spans.n_spans, C.byref(h)))
        d = DeviceSpans(self, h, spans.services)
        d.unique_ids = spans.unique_ids
        d.set_hints(spans.scan_order, spans.hist_form)
        self._reserve_for(d)
        return d

    def _reserve_for(self, d: DeviceSpans):
        """Best effort: the workspace for an ungrouped set's first aggregation
        now (a set that fits HBM while its workspace does not still uploads;
        its aggregation then reports the shortage)."""
        try:
            self.reserve_grouping(d.n_spans)
        except L.AnomodError as e:
            if "ENOMEM" not in str(e):
                raise

    def reserve_grouping(self, n_spans: int, both_records: bool = False):
        """Size the context's grouping workspace for an ungrouped set of
        n_spans ahead of its first aggregation (anomod_ctx_reserve_grouping:
        the ~58 B/span of the join path, + 32 B/span with both_records)."""
        self._check(self._lib.anomod_ctx_reserve_grouping(self.handle, n_spans,
                                                          1 if both_records else 0))

    def group(self, spans: DeviceSpans) -> DeviceSpans:
        """Group an ungrouped device span set by trace (segmented radix sort
        on the GPU): traces by mix64(trace_hash), spans in arrival order."""
        h = C.c_void_p()
        self._check(self._lib.anomod_spans_group(self.handle, spans.handle, C.byref(h)))
        return DeviceSpans(self, h, spans.services)

    def shuffle(self, spans: DeviceSpans, seed: int, window_traces: int = 0) -> DeviceSpans:
        """Synthetic arrival order of a grouped set: window_traces = 0 shuffles
        spans inside each trace (stays grouped); W > 0 interleaves the spans
        of every W consecutive traces (ungrouped result)."""
        h = C.c_void_p()
        self._check(self._lib.anomod_spans_shuffle(self.handle, spans.handle, seed, window_traces,
                                                   C.byref(h)))
        d = DeviceSpans(self, h, spans.services)
        if window_traces:  # an ungrouped set: its grouping workspace now, not at the first call
            self._reserve_for(d)
        return d

    def generate(self, spec: SynthSpec, n_traces: int, shard: int = 0) -> DeviceSpans:
        h = C.c_void_p()
        cs = spec.c_struct()
        self._check(self._lib.anomod_spans_generate(self.handle, C.byref(cs), shard, n_traces,
                                                    C.byref(h)))
        return DeviceSpans(self, h, spec.services())

    def edge_aggregate(self, spans: DeviceSpans | SpanSet, with_hist: bool = True) -> EdgeTable:
        """Edge table of a span set.  A host set goes through
        anomod_edge_aggregate_host (pinned staging pipeline into a device set
        the context keeps; the hints learned on the device go back onto the
        host set)."""
        if isinstance(spans, SpanSet):
            table = EdgeTable.empty(spans.services, with_hist)
            cs = table.c_struct()
            soa = spans.soa()
            order, form = C.c_int(spans.scan_order), C.c_int(spans.hist_form)
            self._check(self._lib.anomod_edge_aggregate_host(
                self.handle, C.byref(soa), spans.n_spans, L.ptr(spans.trace_ptr, C.c_uint64),
                spans.n_traces, len(spans.services), 1 if spans.unique_ids else 0,
                C.byref(order), C.byref(form), C.byref(cs)))
            if table.hist is not None:
                table.hist = table.hist.reshape(edge_rows(len(spans.services)), L.HIST_BINS)
            spans.scan_order, spans.hist_form = order.value, form.value
            return table
        # a device set: its hints live on the set itself (libanomod keeps them)
        table = EdgeTable.empty(spans.services, with_hist)
        cs = table.c_struct()
        fn = (self._lib.anomod_edge_aggregate_spans if spans.grouped
              else self._lib.anomod_edge_aggregate_ungrouped)
        self._check(fn(self.handle, spans.handle, len(spans.services), C.byref(cs)))
        if table.hist is not None:
            table.hist = table.hist.reshape(edge_rows(len(spans.services)), L.HIST_BINS)
        return table

    def edge_quantiles_exact(self, spans: DeviceSpans | SpanSet, q_pct=(50, 99)):
        """Exact per-edge order statistics x[(c*q)//100] of the sorted edge
        latencies ([E, len(q_pct)], NaN for empty edges) and the per-edge
        counts: the cross-check of the histogram quantiles (§8a a11)."""
        tmp = None
        if isinstance(spans, SpanSet):
            tmp = spans = self.upload(spans)
        try:
            q = np.ascontiguousarray(q_pct, np.uint32)
            S = len(spans.services)
            E = edge_rows(S)
            out = np.empty((E, q.shape[0]), np.float64)
            cnt = np.empty(E, np.uint64)
            self._check(self._lib.anomod_edge_quantiles_exact(
                self.handle, spans.handle, S, L.ptr(q, C.c_uint32), q.shape[0],
                L.ptr(out, C.c_double), L.ptr(cnt, C.c_uint64)))
            return out, cnt
        finally:
            if tmp is not None:
                tmp.free()

    def trace_structure(self, spans: DeviceSpans | SpanSet,
                        download: bool = True) -> TraceStructure | None:
        """Per-span parent/depth/children and per-trace roots/services
        (the trace-structure HIP kernel).  download=False runs the kernel
        without copying the outputs back (timing)."""
        tmp = None
        if isinstance(spans, SpanSet):
            tmp = spans = self.upload(spans)
        try:
            if not download:
                cs = L.TraceStructC(len(spans.services))
                self._check(self._lib.anomod_trace_structure_spans(self.handle, spans.handle,
                                                                   C.byref(cs)))
                return None
            ts = TraceStructure.empty(spans.services, spans.n_spans, spans.n_traces)
            cs = ts.c_struct()
            self._check(self._lib.anomod_trace_structure_spans(self.handle, spans.handle,
                                                               C.byref(cs)))
            return ts
        finally:
            if tmp is not None:
                tmp.free()

    def segment_summary(self, seg) -> dict:
        """analyze_trace_patterns over a SegmentSet (segment-summary kernel)."""
        from .segments import segment_summary
        return segment_summary(self, seg)

    # -- metric series
    def ewma_z(self, X: np.ndarray, alpha: float, W: int, eps: float = 1e-12) -> np.ndarray:
        X = np.ascontiguousarray(X, dtype=np.float32)
        T, S = X.shape
        if T % W:
            raise ValueError(f"T={T} must be a multiple of W={W}")
        Z = np.empty((T // W, S), np.float32)
        if T == 0 or S == 0:
            return Z
        self._check(self._lib.anomod_ewma_z(self.handle, L.ptr(X, C.c_float), T, S, alpha, W,
                                            eps, L.ptr(Z, C.c_float)))
        return Z

    # -- ranking
    def pagerank(self, row_ptr, col, w, p, alpha=0.85, iters=100, tol=1e-10):
        row_ptr = np.ascontiguousarray(row_ptr, np.uint32)
        col = np.ascontiguousarray(col, np.uint32)
        w = np.ascontiguousarray(w, np.float32)
        p = np.ascontiguousarray(p, np.float64)
        N = row_ptr.shape[0] - 1
        x = np.empty(N, np.float64)
        done = C.c_uint32()
        if col.size == 0:  # keep the pointers valid for an edgeless graph
            col, w = np.zeros(1, np.uint32), np.zeros(1, np.float32)
        self._check(self._lib.anomod_pagerank(self.handle, L.ptr(row_ptr, C.c_uint32),
                                              L.ptr(col, C.c_uint32), L.ptr(w, C.c_float), N,
                                              L.ptr(p, C.c_double), alpha, iters, tol,
                                              L.ptr(x, C.c_double), C.byref(done)))
        return x, done.value


def synth_graph_csr(N: int, mean_degree: int = 10, seed: int = 11):
    """Host CSR (row_ptr u32, col u32, w f32) of the synthetic config-5 graph
    DeviceGraph(synthetic=(N, mean_degree, seed)) solves."""
    lib = L.lib()
    nnz = C.c_uint64()
    nul32 = C.cast(None, C.POINTER(C.c_uint32))
    L.check(lib.anomod_graph_synthetic_csr(N, mean_degree, seed, nul32, nul32,
                                           C.cast(None, C.POINTER(C.c_float)), 0, C.byref(nnz)))
    row_ptr = np.empty(N + 1, np.uint32)
    col = np.empty(max(1, nnz.value), np.uint32)
    w = np.empty(max(1, nnz.value), np.float32)
    L.check(lib.anomod_graph_synthetic_csr(N, mean_degree, seed, L.ptr(row_ptr, C.c_uint32),
                                           L.ptr(col, C.c_uint32), L.ptr(w, C.c_float),
                                           col.shape[0], C.byref(nnz)))
    return row_ptr, col[:nnz.value], w[:nnz.value]


class DeviceGraph:
    """A CSR graph resident in HBM for repeated PageRank solves."""

    def __init__(self, ctx: Context, row_ptr=None, col=None, w=None, *, synthetic=None):
        self.ctx = ctx
        h = C.c_void_p()
        lib = L.lib()
        if synthetic is not None:
            N, deg, seed = synthetic
            ctx._check(lib.anomod_graph_synthetic(ctx.handle, N, deg, seed, C.byref(h)))
        else:
            row_ptr = np.ascontiguousarray(row_ptr, np.uint32)
            col = np.ascontiguousarray(col, np.uint32)
            w = np.ascontiguousarray(w, np.float32)
            ctx._check(lib.anomod_graph_create(ctx.handle, L.ptr(row_ptr, C.c_uint32),
                                               L.ptr(col, C.c_uint32), L.ptr(w, C.c_float),
                                               row_ptr.shape[0] - 1, C.byref(h)))
        self.handle = h
        n, nnz = C.c_uint32(), C.c_uint64()
        L.check(lib.anomod_graph_info(h, C.byref(n), C.byref(nnz)))
        self.N, self.nnz = n.value, nnz.value

    def pagerank(self, p, alpha=0.85, iters=100, tol=0.0):
        p = np.ascontiguousarray(p, np.float64)
        x = np.empty(self.N, np.float64)
        done = C.c_uint32()
        self.ctx._check(L.lib().anomod_graph_pagerank(self.ctx.handle, self.handle,
                                                      L.ptr(p, C.c_double), alpha, iters, tol,
                                                      L.ptr(x, C.c_double), C.byref(done)))
        return x, done.value

    PATHS = {1: "graph", 2: "readback", 3: "persistent"}

    def last_solve(self) -> tuple[str, int]:
        """(path of the last pagerank() / pagerank_batch() solve, persistent-
        launch fallbacks so far); the path is "graph" / "readback" /
        "persistent" (a per-launch batch reports "graph" for fixed iterations,
        "readback" in tolerance mode), with a
        "fallback:" prefix when a persistent launch timed out at its grid
        barrier and the solve was rerun per launch."""
        path, fb = C.c_uint32(), C.c_uint32()
        L.check(L.lib().anomod_graph_last_solve(self.handle, C.byref(path), C.byref(fb)))
        name = self.PATHS.get(path.value & 3, "none")
        return ("fallback:" + name if path.value & 4 else name), fb.value

    def pagerank_sharded(self, p, alpha=0.85, iters=100, tol=0.0, virtual_shards=0):
        """Row-sharded solve: over the ranks of the attached RCCL communicator,
        or over ``virtual_shards`` row shards on this device when none is
        attached.  Returns the whole vector on every rank."""
        p = np.ascontiguousarray(p, np.float64)
        x = np.empty(self.N, np.float64)
        done = C.c_uint32()
        self.ctx._check(L.lib().anomod_graph_pagerank_sharded(
            self.ctx.handle, self.handle, L.ptr(p, C.c_double), alpha, iters, tol,
            virtual_shards, L.ptr(x, C.c_double), C.byref(done)))
        return x, done.value

    def pagerank_batch(self, P, alpha=0.85, iters=100, tol=0.0):
        """K personalizations ([K, N]) in one batched solve -> x [K, N]."""
        P = np.ascontiguousarray(np.atleast_2d(P), np.float64)
        K = P.shape[0]
        X = np.empty((K, self.N), np.float64)
        done = C.c_uint32()
        self.ctx._check(L.lib().anomod_graph_pagerank_batch(
            self.ctx.handle, self.handle, L.ptr(P, C.c_double), K, alpha, iters, tol,
            L.ptr(X, C.c_double), C.byref(done)))
        return X, done.value

    def free(self):
        if self.handle:
            L.lib().anomod_graph_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class DeviceSeries:
    """A [T][S] metric matrix resident in HBM with carried EWMA state."""

    def __init__(self, ctx: Context, T: int, S: int):
        self.ctx, self.T, self.S = ctx, T, S
        h = C.c_void_p()
        ctx._check(L.lib().anomod_series_create(ctx.handle, T, S, C.byref(h)))
        self.handle = h

    def upload(self, X: np.ndarray):
        X = np.ascontiguousarray(X, np.float32)
        assert X.shape == (self.T, self.S)
        self.ctx._check(L.lib().anomod_series_upload(self.ctx.handle, self.handle,
                                                     L.ptr(X, C.c_float)))

    def fill_synthetic(self, seed: int, t0: int = 0):
        self.ctx._check(L.lib().anomod_series_fill_synthetic(self.ctx.handle, self.handle,
                                                             seed, t0))

    def reset_state(self):
        self.ctx._check(L.lib().anomod_series_reset_state(self.ctx.handle, self.handle))

    def download(self) -> np.ndarray:
        """The resident matrix as host rows X[T][S]."""
        X = np.empty((self.T, self.S), np.float32)
        self.ctx._check(L.lib().anomod_series_download(self.ctx.handle, self.handle,
                                                       L.ptr(X, C.c_float)))
        return X

    def ewma_z(self, alpha: float, W: int, eps: float = 1e-12, download: bool = True):
        Z = np.empty((self.T // W, self.S), np.float32) if download else None
        self.ctx._check(L.lib().anomod_series_ewma_z(
            self.ctx.handle, self.handle, alpha, W, eps,
            L.ptr(Z, C.c_float) if Z is not None else C.cast(None, C.POINTER(C.c_float))))
        return Z

    def free(self):
        if self.handle:
            L.lib().anomod_series_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
