"""Decoders: the dataset's file formats -> columnar SpanSet / metric matrix.

Each decoder restates, column by column, the per-span rules of the reference
collector that wrote the file (paths relative to the reference root):

* Jaeger ``/api/traces`` dumps (SN_data/trace_data/*/all_traces.json) —
  SN_collection-scripts/Dataset/trace_data/jaeger_to_csv.py:21-90.
* SkyWalking raw GraphQL span lists and the collector payload
  (TT_data/trace_data/*/*_skywalking_traces_*.json) —
  TT_collection-scripts/T-Dataset/trace_collector.py:401-481, 536-578.
* Prometheus CSVs — fetch_prometheus_metrics.py:47-67 (SN, one file per
  query) and metric_collector.py:427-467 (TT long format).
"""
from __future__ import annotations

import csv
import ctypes as C
import json
import math
import mmap
import os
import re
from dataclasses import dataclass
from datetime import datetime
from pathlib import Path
from typing import Iterable

import numpy as np
import xxhash

from . import _lib as L
from .spans import SpanSet

U32_MAX = 0xFFFFFFFF
ORPHAN_ID = 0xFFFFFFFFFFFFFFFF  # a parent id no dense local id can equal


def hash64(s: str) -> int:
    """Stable 64-bit id of a string (never 0): xxh64, seed 0 — the hash of the
    native decoders (anomod_hash64)."""
    return xxhash.xxh64_intdigest(s.encode("utf-8", "surrogatepass")) or 1


_HEX_ID = re.compile(r"[0-9a-fA-F]{1,16}")


def jaeger_id(s) -> int:
    """Jaeger spanID -> u64: its value when it is 1-16 hex digits and not 0,
    else xxh64 | 2^63; '' -> 0."""
    if s is None or s == "":
        return 0
    s = str(s)
    if _HEX_ID.fullmatch(s):
        v = int(s, 16)
        if v != 0:
            return v
    return hash64(s) | (1 << 63)


def _clamp_u32(v) -> int:
    try:
        v = int(v)
    except (TypeError, ValueError):
        return 0
    return 0 if v < 0 else U32_MAX if v > U32_MAX else v


def _truthy_error(v) -> bool:
    return v is True or (isinstance(v, str) and v.lower() == "true")


def _status_ge_500(v) -> bool:
    try:
        return int(v) >= 500
    except (TypeError, ValueError):
        return False


# --------------------------------------------------------------------------
# Jaeger (SN)
# --------------------------------------------------------------------------

def jaeger_span_rows(doc: dict) -> Iterable[tuple]:
    """(trace_id, span_id, parent_span_id, service, duration_us, tags) per span,
    in file order — the columns jaeger_to_csv.py:76-90 writes."""
    for trace in doc.get("data", []) or []:
        trace_id = trace.get("traceID", "")
        proc = {pid: (info or {}).get("serviceName", "")
                for pid, info in (trace.get("processes", {}) or {}).items()}
        for span in trace.get("spans", []) or []:
            parent = ""
            for ref in span.get("references", []) or []:
                if ref.get("refType") == "CHILD_OF":  # first CHILD_OF wins (:35-38)
                    parent = ref.get("spanID", "")
                    break
            tags = {}
            for tag in span.get("tags", []) or []:
                tags[tag.get("key", "")] = tag.get("value", "")  # last key wins (:58)
            yield (trace_id, span.get("spanID", ""), parent,
                   proc.get(span.get("processID", ""), ""), span.get("duration", 0), tags)


def decode_jaeger(doc: dict, services: list[str] | None = None) -> SpanSet:
    """Jaeger dump -> SpanSet.  Error flag: tags['error'] true or
    http.status_code >= 500 (tags as kept at jaeger_to_csv.py:55-67)."""
    rows = []
    trace_ptr = [0]
    trace_ids = []
    for trace in doc.get("data", []) or []:
        rows.extend(jaeger_span_rows({"data": [trace]}))
        trace_ids.append(trace.get("traceID", ""))
        trace_ptr.append(len(rows))
    names = sorted({r[3] for r in rows}) if services is None else list(services)
    index = {s: i for i, s in enumerate(names)}
    n = len(rows)
    th = np.empty(n, np.uint64)
    sid = np.empty(n, np.uint64)
    pid = np.empty(n, np.uint64)
    svc = np.empty(n, np.uint16)
    flg = np.zeros(n, np.uint16)
    dur = np.empty(n, np.uint32)
    tcache: dict[str, int] = {}
    for i, (tid, s, p, service, d, tags) in enumerate(rows):
        h = tcache.get(tid)
        if h is None:
            h = tcache[tid] = hash64(str(tid))
        th[i] = h
        sid[i] = jaeger_id(s)
        pid[i] = jaeger_id(p)
        if service not in index:
            raise KeyError(f"service {service!r} not in the service list")
        svc[i] = index[service]
        dur[i] = _clamp_u32(d)
        if _truthy_error(tags.get("error")) or _status_ge_500(tags.get("http.status_code")):
            flg[i] = 1
    return SpanSet(names, np.asarray(trace_ptr, np.uint64), th, sid, pid, svc, flg, dur,
                   trace_ids)


def merge_jaeger_dumps(dumps: Iterable[dict]) -> dict:
    """Union of per-service /api/traces dumps as collect_trace.sh:54-58 builds
    it: ``.[0].data + .[1].data | unique_by(.traceID)`` per service — sorted
    by traceID, the first occurrence of each id kept (jq is not installed
    here, so this restatement is unpinned against jq itself)."""
    merged: list = []
    for d in dumps:
        data = (d or {}).get("data") or []
        if not data:
            continue
        seen: dict = {}
        for tr in merged + list(data):
            seen.setdefault(tr.get("traceID"), tr)
        # jq orders null before strings
        merged = [seen[k] for k in sorted(seen, key=lambda k: (k is not None, str(k)))]
    return {"data": merged}


# --------------------------------------------------------------------------
# SkyWalking (TT)
# --------------------------------------------------------------------------

def skywalking_parents(spans: list[dict]) -> tuple[list[str], list[str | None], list[dict]]:
    """Node ids and parent node ids of one trace's raw GraphQL spans, as
    _build_span_records resolves them (trace_collector.py:408-437): spans
    without segmentId/spanId are dropped; parent = same segment when
    parentSpanId is an int >= 0, else refs[0]."""
    kept, nodes, parents = [], [], []
    for span in spans:
        seg, sp = span.get("segmentId"), span.get("spanId")
        if seg is None or sp is None:
            continue
        kept.append(span)
        nodes.append(f"{seg}:{sp}")
    for span in kept:
        parent = None
        psid = span.get("parentSpanId", -1)
        # bool is an int in Python, exactly as in the reference's isinstance test
        if isinstance(psid, int) and psid >= 0:
            parent = f"{span.get('segmentId')}:{psid}"
        else:
            refs = span.get("refs") or []
            if refs:
                ps, pp = refs[0].get("parentSegmentId"), refs[0].get("parentSpanId")
                if ps is not None and pp is not None:
                    parent = f"{ps}:{pp}"
        parents.append(parent)
    return nodes, parents, kept


@dataclass
class _TraceRows:
    trace_id: str
    nodes: list
    parents: list
    services: list
    dur_us: list
    errors: list


def _dense_ids(nodes: list[str], parents: list) -> tuple[list[int], list[int]]:
    first: dict[str, int] = {}
    for i, n in enumerate(nodes):
        first.setdefault(n, i + 1)
    sids = [first[n] for n in nodes]
    pids = [0 if p is None else first.get(p, ORPHAN_ID) for p in parents]
    return sids, pids


def _build(traces: list[_TraceRows], services: list[str] | None) -> SpanSet:
    names = (sorted({s for t in traces for s in t.services}) if services is None
             else list(services))
    index = {s: i for i, s in enumerate(names)}
    th, sid, pid, svc, flg, dur, ptr, ids = [], [], [], [], [], [], [0], []
    for t in traces:
        s_ids, p_ids = _dense_ids(t.nodes, t.parents)
        h = hash64(str(t.trace_id))
        th.extend([h] * len(t.nodes))
        sid.extend(s_ids)
        pid.extend(p_ids)
        svc.extend(index[s] for s in t.services)
        flg.extend(1 if e else 0 for e in t.errors)
        dur.extend(t.dur_us)
        ptr.append(len(sid))
        ids.append(t.trace_id)
    return SpanSet(names, np.asarray(ptr, np.uint64), np.asarray(th, np.uint64),
                   np.asarray(sid, np.uint64), np.asarray(pid, np.uint64),
                   np.asarray(svc, np.uint16), np.asarray(flg, np.uint16),
                   np.asarray(dur, np.uint32), ids)


def _ms_to_us(start, end) -> int:
    """duration_ms = max(0, end - start) (trace_collector.py:87) in microseconds."""
    try:
        d = int(end or 0) - int(start or 0)
    except (TypeError, ValueError):
        d = 0
    return _clamp_u32(max(0, d) * 1000)


def decode_skywalking_raw(traces: Iterable[list[dict]], services: list[str] | None = None
                          ) -> SpanSet:
    """Raw GraphQL span lists (one list per trace, the input of
    _build_span_records) -> SpanSet."""
    rows = []
    for spans in traces:
        nodes, parents, kept = skywalking_parents(list(spans))
        if not kept:
            continue  # "no usable span records" (trace_collector.py:532-534)
        rows.append(_TraceRows(
            str(kept[0].get("traceId") or ""), nodes, parents,
            [s.get("serviceCode") or "" for s in kept],
            [_ms_to_us(s.get("startTime", 0), s.get("endTime", 0)) for s in kept],
            [bool(s.get("isError", False)) for s in kept]))
    return _build(rows, services)


def decode_skywalking_payload(payload: dict, services: list[str] | None = None) -> SpanSet:
    """Collector payload ({metadata, traces:[{summary, spans:[SpanRecord]}]},
    trace_collector.py:564-578) -> SpanSet, using the node/parent ids the
    collector already resolved (SpanRecord.to_dict, :97-123)."""
    rows = []
    for tr in payload.get("traces", []) or []:
        spans = tr.get("spans") or []
        if not spans:
            continue
        tid = (tr.get("summary") or {}).get("trace_id") or spans[0].get("trace_id") or ""
        rows.append(_TraceRows(
            str(tid), [s.get("node_id") for s in spans], [s.get("parent_node_id") for s in spans],
            [s.get("service_code") or "" for s in spans],
            [_ms_to_us(s.get("start_timestamp_ms", 0), s.get("end_timestamp_ms", 0))
             for s in spans],
            [bool(s.get("is_error", False)) for s in spans]))
    return _build(rows, services)


# --------------------------------------------------------------------------
# Prometheus metrics
# --------------------------------------------------------------------------

@dataclass
class MetricMatrix:
    """Time-major metric matrix X[T][S] (NaN = no sample) on a regular grid."""

    X: np.ndarray              # f32 [T, S]
    timestamps: np.ndarray     # f64 [T] epoch seconds
    series: list[tuple]        # [S] (metric_name, ((label, value), ...))

    @property
    def T(self) -> int:
        return int(self.X.shape[0])

    @property
    def S(self) -> int:
        return int(self.X.shape[1])

    def pad_to_multiple(self, W: int) -> "MetricMatrix":
        T = self.T
        Tp = ((T + W - 1) // W) * W if T else 0
        if Tp == T:
            return self
        X = np.full((Tp, self.S), np.nan, np.float32)
        X[:T] = self.X
        ts = np.concatenate([self.timestamps, self.timestamps[-1:] + np.arange(1, Tp - T + 1)])
        return MetricMatrix(X, ts, self.series)


def _to_matrix(samples: dict, ts_set: set) -> MetricMatrix:
    keys = sorted(samples, key=lambda k: (k[0], k[1]))
    ts = np.asarray(sorted(ts_set), np.float64)
    col = {t: i for i, t in enumerate(ts.tolist())}
    X = np.full((len(ts), len(keys)), np.nan, np.float32)
    for j, k in enumerate(keys):
        for t, v in samples[k].items():
            X[col[t], j] = v
    return MetricMatrix(X, ts, keys)


def decode_metric_long_csv(path_or_lines) -> MetricMatrix:
    """TT long CSV (metric_name,timestamp,datetime,value,<sorted labels>;
    metric_collector.py:453-467).  Series key = (metric_name, non-empty label
    pairs).  Empty value ('NaN' -> None -> '' at :435) = missing.  The CSV
    repeats three metrics (key_metrics has 36 entries, 33 unique, :37-109), so
    rows are de-duplicated on (series, timestamp), first occurrence kept."""
    if isinstance(path_or_lines, (str, Path)):
        fh = open(path_or_lines, newline="", encoding="utf-8")
    else:
        fh = path_or_lines
    samples: dict = {}
    ts_set: set = set()
    try:
        rd = csv.DictReader(fh)
        fixed = {"metric_name", "timestamp", "datetime", "value"}
        for row in rd:
            labels = tuple(sorted((k, v) for k, v in row.items() if k not in fixed and v))
            key = (row["metric_name"], labels)
            t = float(row["timestamp"])
            ts_set.add(t)
            d = samples.setdefault(key, {})
            if t in d:
                continue
            v = row["value"]
            d[t] = float(v) if v not in ("", None) else math.nan
    finally:
        if isinstance(path_or_lines, (str, Path)):
            fh.close()
    return _to_matrix(samples, ts_set)


def decode_prometheus_csv_dir(directory) -> MetricMatrix:
    """SN metric directory: one CSV per query (fetch_prometheus_metrics.py:57-67:
    timestamp = local datetime string, value, metric = label string).  Series
    key = (query file stem, metric label string)."""
    samples: dict = {}
    ts_set: set = set()
    for path in sorted(Path(directory).glob("*.csv")):
        with open(path, newline="", encoding="utf-8") as fh:
            for row in csv.DictReader(fh):
                t = datetime.fromisoformat(row["timestamp"]).timestamp()
                ts_set.add(t)
                key = (path.stem, (("metric", row.get("metric", "")),))
                d = samples.setdefault(key, {})
                if t not in d:
                    v = row.get("value", "")
                    d[t] = float(v) if v not in ("", None) else math.nan
    return _to_matrix(samples, ts_set)


def _series_packed(lib, h, S: int):
    """Every series' (name, labels) from one anomod_metrics_series_packed call
    (a per-string call per name and label cost ~25 ms for the 5 850 series of
    a TrainTicket experiment); None when the strings do not split cleanly."""
    need = C.c_uint64()
    nl = np.zeros(max(1, S), np.uint32)
    L.check(lib.anomod_metrics_series_packed(h, None, 0, L.ptr(nl, C.c_uint32), C.byref(need)))
    buf = C.create_string_buffer(max(1, need.value))
    L.check(lib.anomod_metrics_series_packed(h, buf, need.value, L.ptr(nl, C.c_uint32),
                                             C.byref(need)))
    parts = buf.raw[:need.value].decode().split("\0")
    counts = nl[:S]
    if len(parts) != S + 2 * int(counts.sum()) + 1:
        return None
    if S and (counts == counts[0]).all():  # the usual case: one label set per file
        c = int(counts[0])
        st = 1 + 2 * c
        pairs = zip(*[zip(parts[1 + 2 * j:-1:st], parts[2 + 2 * j:-1:st]) for j in range(c)])
        return list(zip(parts[0:-1:st], pairs)) if c else [(n, ()) for n in parts[0:-1:st]]
    series, i = [], 0
    for n in counts.tolist():
        series.append((parts[i], tuple((parts[i + 1 + 2 * j], parts[i + 2 + 2 * j])
                                       for j in range(n))))
        i += 1 + 2 * n
    return series


def _metrics_from_handle(h) -> MetricMatrix:
    lib = L.lib()
    try:
        T, S = C.c_uint64(), C.c_uint64()
        L.check(lib.anomod_metrics_info(h, C.byref(T), C.byref(S)))
        X = np.empty((T.value, S.value), np.float32)
        ts = np.empty(T.value, np.float64)
        L.check(lib.anomod_metrics_matrix(h, L.ptr(X, C.c_float), L.ptr(ts, C.c_double)))
        series = _series_packed(lib, h, S.value)
        if series is None:  # a name holding a NUL byte: one call per string
            series = []
            val = C.c_char_p()
            for s in range(S.value):
                name = lib.anomod_metrics_series_name(h, s).decode()
                labels = []
                for j in range(lib.anomod_metrics_series_nlabels(h, s)):
                    k = lib.anomod_metrics_series_label(h, s, j, C.byref(val))
                    labels.append((k.decode(), val.value.decode()))
                series.append((name, tuple(labels)))
    finally:
        lib.anomod_metrics_free(h)
    return MetricMatrix(X, ts, series)


class MappedFile:
    """A file's bytes for the native decoders without a copy: a read-only
    shared mapping (PROT_READ, so the pages stay the page cache's own — a
    private writable mapping would copy every page at fault time).  Slicing
    gives bytes; ``as_arg()`` is the address for a ``const char*`` parameter
    (valid while this object lives)."""

    def __init__(self, path):
        with open(path, "rb") as fh:
            self.size = os.fstat(fh.fileno()).st_size
            self._mm = (mmap.mmap(fh.fileno(), self.size, prot=mmap.PROT_READ)
                        if self.size else None)
        self._view = (np.frombuffer(self._mm, np.uint8) if self._mm is not None
                      else np.zeros(0, np.uint8))

    def __len__(self) -> int:
        return self.size

    def __getitem__(self, sl) -> bytes:
        return self._mm[sl] if self._mm is not None else b""[sl]

    def as_arg(self):
        if self._mm is None:
            return b""
        return C.cast(C.c_void_p(self._view.ctypes.data), C.c_char_p)


def map_file(path) -> MappedFile:
    """A file mapped read-only for the native decoders (see MappedFile)."""
    return MappedFile(path)


def decode_metric_long_csv_native(path_or_bytes) -> MetricMatrix:
    """decode_metric_long_csv in libanomod (csrc/metrics_decode.cpp): the
    same matrix, without a Python dict per row.  A path is mapped, not read
    (anomod_decode_metric_long_csv_file)."""
    if isinstance(path_or_bytes, bytearray):
        data = bytes(path_or_bytes)
    elif isinstance(path_or_bytes, bytes):
        data = path_or_bytes
    else:  # mapped by the library: its parser threads fault their own pieces
        h = C.c_void_p()
        L.check(L.lib().anomod_decode_metric_long_csv_file(os.fsencode(path_or_bytes),
                                                           C.byref(h)))
        return _metrics_from_handle(h)
    h = C.c_void_p()
    L.check(L.lib().anomod_decode_metric_long_csv(data, len(data), C.byref(h)))
    return _metrics_from_handle(h)


def decode_prometheus_csv_dir_native(directory) -> MetricMatrix:
    """decode_prometheus_csv_dir in libanomod: one CSV per query, files in
    sorted path order, series = (file stem, 'metric' column)."""
    paths = sorted(Path(directory).glob("*.csv"))
    blobs = [p.read_bytes() for p in paths]
    n = len(paths)
    data = (C.c_char_p * max(1, n))(*blobs)
    lens = (C.c_uint64 * max(1, n))(*[len(b) for b in blobs])
    stems = (C.c_char_p * max(1, n))(*[p.stem.encode() for p in paths])
    h = C.c_void_p()
    L.check(L.lib().anomod_decode_prometheus_csvs(data, lens, stems, n, C.byref(h)))
    return _metrics_from_handle(h)


# --------------------------------------------------------------------------
# Native decoders (libanomod, csrc/decode.cpp): same columns as the Python
# decoders above, without a Python object per span
# --------------------------------------------------------------------------

def decode_native(data: "bytes | MappedFile", kind: str, services: list[str] | None = None) -> SpanSet:
    """A Jaeger dump (kind 'jaeger') or a SkyWalking collector payload
    (kind 'skywalking') -> SpanSet, parsed by the native decoder."""
    lib = L.lib()
    fn = {"jaeger": lib.anomod_decode_jaeger, "skywalking": lib.anomod_decode_skywalking}[kind]
    names = None
    if services is not None:
        names = (C.c_char_p * max(1, len(services)))(*[s.encode() for s in services])
    h = C.c_void_p()
    arg = data.as_arg() if isinstance(data, MappedFile) else data
    L.check(fn(arg, len(data), names, 0 if services is None else len(services), C.byref(h)))
    try:
        ns, nt, nsv = C.c_uint64(), C.c_uint64(), C.c_uint32()
        L.check(lib.anomod_decoded_info(h, C.byref(ns), C.byref(nt), C.byref(nsv)))
        n = ns.value
        arr = dict(trace_hash=np.empty(n, np.uint64), span_id=np.empty(n, np.uint64),
                   parent_span_id=np.empty(n, np.uint64), svc=np.empty(n, np.uint16),
                   flags=np.empty(n, np.uint16), dur_us=np.empty(n, np.uint32))
        ptr = np.empty(nt.value + 1, np.uint64)
        soa = L.SpanSoA(*[L.ptr(arr[k], t) for k, t in (
            ("trace_hash", C.c_uint64), ("span_id", C.c_uint64), ("parent_span_id", C.c_uint64),
            ("svc", C.c_uint16), ("flags", C.c_uint16), ("dur_us", C.c_uint32))])
        L.check(lib.anomod_decoded_columns(h, C.byref(soa), L.ptr(ptr, C.c_uint64)))
        svcs = [lib.anomod_decoded_service(h, i).decode() for i in range(nsv.value)]
        uniq = C.c_int()
        L.check(lib.anomod_decoded_unique_ids(h, C.byref(uniq)))
    finally:
        lib.anomod_decoded_free(h)
    # the decoder checked every trace's ids exactly while decoding
    return SpanSet(svcs, ptr, **arr, unique_ids=bool(uniq.value))


def _first_key(data: bytes) -> str | None:
    m = re.match(rb'\s*\{\s*"((?:[^"\\]|\\.)*)"', data[:4096])
    return m.group(1).decode("utf-8", "replace") if m else None


def load_trace_file(path, services: list[str] | None = None) -> SpanSet:
    """A trace file of the dataset -> SpanSet: Jaeger dumps ({"data": ...})
    and collector payloads ({"metadata": ..., "traces": ...}) go through the
    native decoder; anything else (raw GraphQL span lists) through the
    Python decoders.  The set's unique_ids is checked exactly (by the native
    decoder while it decodes, else on the columns)."""
    data = map_file(path)
    key = _first_key(data[:4096])
    if key == "data":
        return decode_native(data, "jaeger", services)
    if key in ("metadata", "traces"):
        return decode_native(data, "skywalking", services)
    spans = _load_trace_file_py(data, path, services)
    spans.check_unique_ids()
    return spans


def _load_trace_file_py(data, path, services: list[str] | None = None) -> SpanSet:
    doc = json.loads(data[:])
    if isinstance(doc, dict) and "traces" in doc:
        return decode_skywalking_payload(doc, services)
    if isinstance(doc, dict) and "data" in doc:
        return decode_jaeger(doc, services)
    if isinstance(doc, list):
        return decode_skywalking_raw(doc, services)
    raise ValueError(f"{path}: not a Jaeger dump or SkyWalking payload")


def load_json(path) -> dict:
    with open(path, encoding="utf-8") as fh:
        return json.load(fh)
