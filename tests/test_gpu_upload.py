"""GPU: the host -> device span upload (csrc/upload.hip).  Direct (default):
columns of at least a piece registered for the call and copied from the
caller's pages, svc | flags copied as two u16 columns and packed on the
device, smaller items from pageable memory (svc | flags packed on the host).
Bounce (a refused registration, or ANOMOD_UPLOAD_DIRECT=0): the columns cut
into 8-MiB pieces (2 Mi packed svc|flags elements) dealt to W worker threads
with their own streams and pinned buffers.  Every column must arrive
bit-equal whatever the path, the worker count and wherever the piece cuts
fall, the largest service must come from whichever packing ran, and the
context's reused host-call set (anomod_edge_aggregate_host) must never show
a previous call's spans."""
import numpy as np
import pytest

import anomod
from oracle import native

from test_gpu_edge import _random_spanset, assert_table_equal

pytestmark = pytest.mark.gpu

PIECE_U64 = (8 << 20) // 8  # u64 elements per piece
PIECE_PACKED = (8 << 20) // 4  # svc|flags elements per piece


def _flat_spanset(rng, n, S=12, trace_len=7):
    """n spans in traces of trace_len (the last one shorter), random columns."""
    lens = [trace_len] * (n // trace_len) + ([n % trace_len] if n % trace_len else [])
    ptr = np.zeros(len(lens) + 1, np.uint64)
    np.cumsum(lens, out=ptr[1:])
    sid = rng.integers(1, 2**63, n, dtype=np.uint64)
    pid = rng.integers(0, 2**63, n, dtype=np.uint64)
    th = rng.integers(0, 2**63, n, dtype=np.uint64)
    svc = rng.integers(0, S, n).astype(np.uint16)
    flg = rng.integers(0, 1 << 16, n).astype(np.uint16)
    dur = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    return anomod.SpanSet([f"s{i}" for i in range(S)], ptr, th, sid, pid, svc, flg, dur)


def _assert_columns_equal(a: anomod.SpanSet, b: anomod.SpanSet):
    for k in ("trace_ptr", "trace_hash", "span_id", "parent_span_id", "svc", "flags", "dur_us"):
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k), err_msg=k)


@pytest.mark.parametrize("threads,direct", [("1", "0"), ("3", "0"), ("8", "0"), ("8", "1")])
def test_upload_roundtrip_piece_cuts(monkeypatch, threads, direct):
    """Sizes around the piece cuts of both item kinds (u64 columns: 2^20
    elements a piece; packed svc|flags: 2^21), one span, and none — through a
    fresh context whose bounce pipeline has `threads` workers (direct "0"),
    or the direct path (small items pageable, large ones registered)."""
    monkeypatch.setenv("ANOMOD_UPLOAD_THREADS", threads)
    monkeypatch.setenv("ANOMOD_UPLOAD_DIRECT", direct)
    rng = np.random.default_rng(int(threads))
    with anomod.Context(0) as c:
        for n in (0, 1, PIECE_U64 - 1, PIECE_U64 + 1, PIECE_PACKED + 3, 3 * PIECE_U64 + 5):
            sp = _flat_spanset(rng, n)
            dev = c.upload(sp)
            _assert_columns_equal(dev.download(), sp)
            dev.free()


@pytest.mark.parametrize("direct", ["1", "0"])
def test_upload_max_service_from_packing(ctx, monkeypatch, direct):
    """The set's largest service comes from the packing — the device pack
    kernel (direct) or the workers' pass (bounce): a set whose one
    out-of-range service sits in the last piece of a multi-piece upload is
    refused by the aggregation (not silently indexed past the table); the
    same set in range aggregates oracle-equal.  A small set (host packing)
    likewise."""
    monkeypatch.setenv("ANOMOD_UPLOAD_DIRECT", direct)
    small = _random_spanset(np.random.default_rng(6), 12, 50, 9)
    sbad = small.svc.copy()
    sbad[-1] = 12
    with pytest.raises(anomod.AnomodError, match="service index 12"):
        ctx.edge_aggregate(anomod.SpanSet(small.services, small.trace_ptr, small.trace_hash,
                                          small.span_id, small.parent_span_id, sbad,
                                          small.flags, small.dur_us))
    rng = np.random.default_rng(5)
    sp = _random_spanset(rng, 12, PIECE_PACKED // 3, 9)
    n = sp.n_spans
    assert n > PIECE_PACKED
    bad_svc = sp.svc.copy()
    bad_svc[n - 1] = 12  # == n_services
    bad = anomod.SpanSet(sp.services, sp.trace_ptr, sp.trace_hash, sp.span_id,
                         sp.parent_span_id, bad_svc, sp.flags, sp.dur_us)
    with pytest.raises(anomod.AnomodError, match="service index 12"):
        ctx.edge_aggregate(bad)
    dev = ctx.upload(bad)
    with pytest.raises(anomod.AnomodError, match="service index 12"):
        ctx.edge_aggregate(dev)
    dev.free()
    assert_table_equal(ctx.edge_aggregate(sp), native.edge_aggregate(sp))


def test_host_calls_reuse_the_context_set(ctx):
    """anomod_edge_aggregate_host keeps one grow-only device set per context:
    a smaller set after a larger one, a larger one after that (the set grows),
    and the first again — each table equal to its own oracle table (nothing
    of a previous call's spans, traces or hints leaks into the next)."""
    rng = np.random.default_rng(17)
    sets = [_random_spanset(rng, 12, 40000, 20, dup=0.01),
            _random_spanset(rng, 12, 3000, 20, dup=0.01),
            _random_spanset(rng, 20, 90000, 20, dup=0.01),
            _random_spanset(rng, 12, 1, 3)]
    refs = [native.edge_aggregate(s) for s in sets]
    for i in (0, 1, 2, 3, 0, 2, 1):
        assert_table_equal(ctx.edge_aggregate(sets[i]), refs[i])


def test_upload_rejects_bad_trace_ptr(ctx):
    rng = np.random.default_rng(3)
    sp = _flat_spanset(rng, 100)
    ptr = sp.trace_ptr.copy()
    ptr[3], ptr[4] = ptr[4], ptr[3]  # not non-decreasing
    bad = anomod.SpanSet(sp.services, ptr, sp.trace_hash, sp.span_id, sp.parent_span_id,
                         sp.svc, sp.flags, sp.dur_us)
    with pytest.raises(anomod.AnomodError, match="non-decreasing"):
        ctx.upload(bad)
    with pytest.raises(anomod.AnomodError, match="non-decreasing"):
        ctx.edge_aggregate(bad)
    over = sp.trace_ptr.copy()
    over[-1] = sp.n_spans + 1
    bad = anomod.SpanSet(sp.services, over, sp.trace_hash, sp.span_id, sp.parent_span_id,
                         sp.svc, sp.flags, sp.dur_us)
    with pytest.raises(anomod.AnomodError):
        ctx.upload(bad)


@pytest.mark.parametrize("direct", ["1", "0"])
def test_upload_direct_and_bounce_columns(monkeypatch, direct):
    """r06: plain columns of >= one piece are registered for the call and
    copied straight from the caller's pages (ANOMOD_UPLOAD_DIRECT=0: all
    through the bounce pipeline).  Columns that share a page (two views of
    one buffer, so the second registration is refused and that column falls
    back to the bounce pipeline), a read-only column and a plain one all
    arrive bit-equal, and repeated calls on the same arrays (registered and
    unregistered each time) too."""
    monkeypatch.setenv("ANOMOD_UPLOAD_DIRECT", direct)
    rng = np.random.default_rng(11)
    n = 3 * PIECE_U64 + 123  # not a page multiple: the two views share a page
    sp = _flat_spanset(rng, n)
    both = np.concatenate([sp.span_id, sp.parent_span_id])
    dur = sp.dur_us.copy()
    dur.flags.writeable = False
    shared = anomod.SpanSet(sp.services, sp.trace_ptr, sp.trace_hash, both[:n], both[n:],
                            sp.svc, sp.flags, dur)
    with anomod.Context(0) as c:
        for _ in range(2):
            dev = c.upload(shared)
            _assert_columns_equal(dev.download(), sp)
            dev.free()
        sp2 = _random_spanset(rng, 12, PIECE_U64 // 4, 9)
        for _ in range(2):
            assert_table_equal(c.edge_aggregate(sp2), native.edge_aggregate(sp2))
