"""GPU parity: grouping of ungrouped span sets (the segmented radix sort,
csrc/group.hip) against the oracle's stable grouping (oracle/spec.py
group_by_trace), and the edge table / trace structure of interleaved input
against the C oracle on the oracle-grouped spans, bit for bit."""
import numpy as np
import pytest

import anomod
from oracle import native, spec

from test_gpu_edge import _random_spanset, assert_table_equal

pytestmark = pytest.mark.gpu

COLS = ("trace_hash", "span_id", "parent_span_id", "svc", "flags", "dur_us")


def _interleave(sp: anomod.SpanSet, rng, mode: str) -> anomod.SpanSet:
    """Arrival orders: 'random' (uniform permutation), 'time' (traces start in
    order, each span lands at its trace's start + a random delay: the
    ES start_time order of enhanced_trace_collector.py:80-90 across
    concurrent traces), 'reverse'."""
    n = sp.n_spans
    if mode == "random":
        order = rng.permutation(n)
    elif mode == "reverse":
        order = np.arange(n)[::-1]
    else:
        t_of = np.repeat(np.arange(sp.n_traces), np.diff(sp.trace_ptr).astype(np.int64))
        when = t_of * 10.0 + rng.exponential(200.0, n)
        order = np.argsort(when, kind="stable")
    return anomod.SpanSet(sp.services, np.zeros(1, np.uint64), sp.trace_hash[order],
                          sp.span_id[order], sp.parent_span_id[order], sp.svc[order],
                          sp.flags[order], sp.dur_us[order])


def _with_trace_hashes(sp: anomod.SpanSet, rng, hashes=None) -> anomod.SpanSet:
    nt = sp.n_traces
    th = rng.integers(0, 2**64, nt, dtype=np.uint64) if hashes is None else hashes
    sp.trace_hash = np.repeat(th, np.diff(sp.trace_ptr).astype(np.int64)).astype(np.uint64)
    return sp


def _oracle_grouped(flat: anomod.SpanSet) -> anomod.SpanSet:
    order, tptr = spec.group_by_trace(flat.trace_hash)
    return flat.take(order, tptr)


def _assert_grouped_equal(got: anomod.SpanSet, want: anomod.SpanSet):
    np.testing.assert_array_equal(got.trace_ptr, want.trace_ptr, err_msg="trace_ptr")
    for k in COLS:
        np.testing.assert_array_equal(getattr(got, k), getattr(want, k), err_msg=k)


@pytest.mark.parametrize("n_traces,max_len,mode", [
    (1, 1, "random"), (3, 5, "reverse"), (200, 12, "random"), (5000, 20, "time"),
    (40000, 12, "random"), (300000, 14, "time"),
])
def test_group_matches_oracle(ctx, n_traces, max_len, mode):
    rng = np.random.default_rng(n_traces + max_len)
    sp = _with_trace_hashes(_random_spanset(rng, 12, n_traces, max_len, dup=0.02), rng)
    flat = _interleave(sp, rng, mode)
    dev = ctx.upload_ungrouped(flat)
    assert not dev.grouped
    g = ctx.group(dev)
    assert g.grouped
    _assert_grouped_equal(g.download(), _oracle_grouped(flat))
    g.free()
    dev.free()


def test_group_empty(ctx):
    sp = anomod.SpanSet(["a"], np.zeros(1, np.uint64), *(np.zeros(0, t) for t in (
        np.uint64, np.uint64, np.uint64, np.uint16, np.uint16, np.uint32)))
    dev = ctx.upload_ungrouped(sp)
    g = ctx.group(dev)
    assert g.n_spans == 0 and g.n_traces == 0
    t = ctx.edge_aggregate(dev)
    assert t.count.sum() == 0


def _unmix64(k: np.ndarray) -> np.ndarray:
    """Inverse of spec.mix64 (hashes with chosen mixed keys)."""
    M = 2**64

    def unxorshift(y, s):
        x = y.copy()
        for _ in range(64 // s + 1):
            x = y ^ (x >> np.uint64(s))
        return x

    z = unxorshift(np.asarray(k, np.uint64), 31)
    z = z * np.uint64(pow(0x94D049BB133111EB, -1, M))
    z = unxorshift(z, 27)
    z = z * np.uint64(pow(0xBF58476D1CE4E5B9, -1, M))
    return unxorshift(z, 30)


def test_mixed_buckets_and_pass_retry(ctx):
    """Traces whose mixed keys share their top 40 bits land in one bucket at
    every pass count below 6: buckets of two or three traces take the
    in-LDS fix-up, a 1800-span mixed bucket exceeds it and forces reruns with
    more radix passes; the output is the same stable grouping."""
    rng = np.random.default_rng(3)
    k = rng.integers(0, 2**64, 10, dtype=np.uint64)
    assert (spec.mix64(_unmix64(k)) == k).all()
    base = rng.integers(0, 2**64, 1, dtype=np.uint64)[0] & np.uint64(0xFFFFFFFFFF000000)
    keys = []
    keys += [base | np.uint64(x) for x in rng.integers(0, 2**24, 3, dtype=np.uint64)]  # big mix
    for _ in range(50):  # pairs sharing 40 top bits elsewhere
        b = rng.integers(0, 2**64, 1, dtype=np.uint64)[0] & np.uint64(0xFFFFFFFFFF000000)
        keys += [b | np.uint64(x) for x in rng.integers(0, 2**24, 2, dtype=np.uint64)]
    keys = np.asarray(keys, np.uint64)
    hashes = _unmix64(keys)
    lens = np.r_[np.full(3, 600), rng.integers(1, 30, len(keys) - 3)]
    sp = _with_trace_hashes(_random_spanset(rng, 12, 0, 0, dup=0.02, lens=lens), rng, hashes)
    extra = _with_trace_hashes(_random_spanset(rng, 12, 2000, 10), rng)
    sp = anomod.SpanSet.concat([sp, extra])
    flat = _interleave(sp, rng, "random")
    g = ctx.group(ctx.upload_ungrouped(flat))
    _assert_grouped_equal(g.download(), _oracle_grouped(flat))


@pytest.mark.parametrize("mode", ["random", "time"])
def test_edge_aggregate_ungrouped_bit_exact(ctx, mode):
    """Interleaved spans with duplicate ids and orphans: the edge table of
    the ungrouped set equals the oracle's on the stably grouped spans (the
    first-match parent rule sees each trace in arrival order)."""
    rng = np.random.default_rng(11)
    sp = _with_trace_hashes(_random_spanset(rng, 12, 30000, 24, dup=0.05), rng)
    big = _with_trace_hashes(_random_spanset(rng, 12, 3, 900, dup=0.05), rng)
    flat = _interleave(anomod.SpanSet.concat([sp, big]), rng, mode)
    dev = ctx.upload_ungrouped(flat)
    assert_table_equal(ctx.edge_aggregate(dev), native.edge_aggregate(_oracle_grouped(flat)))


def test_trace_structure_of_grouped_ungrouped(ctx):
    rng = np.random.default_rng(5)
    sp = _with_trace_hashes(_random_spanset(rng, 20, 8000, 30, dup=0.03), rng)
    flat = _interleave(sp, rng, "time")
    g = ctx.group(ctx.upload_ungrouped(flat))
    got = ctx.trace_structure(g)
    want = native.trace_structure(_oracle_grouped(flat))
    for k in ("parent_pos", "depth", "n_children", "span_flags", "n_roots", "svc_mask"):
        np.testing.assert_array_equal(getattr(got, k), want[k], err_msg=k)


def test_device_shuffles(ctx):
    """Window interleave and in-trace shuffle of a device-generated SN set:
    ungrouped edge table == the oracle on the regrouped download; in-trace
    shuffle keeps trace_ptr and each trace's multiset of spans."""
    spec_ = anomod.SynthSpec("SN", seed=21, p_orphan_ppm=2000)
    dev = ctx.generate(spec_, 60000)
    host = dev.download()
    inter = ctx.shuffle(dev, seed=7, window_traces=4096)
    assert not inter.grouped and inter.n_spans == dev.n_spans
    flat = inter.download()
    assert sorted(flat.span_id.tolist()) == sorted(host.span_id.tolist())
    assert_table_equal(ctx.edge_aggregate(inter), native.edge_aggregate(_oracle_grouped(flat)))
    intra = ctx.shuffle(dev, seed=9, window_traces=0)
    assert intra.grouped
    ih = intra.download()
    np.testing.assert_array_equal(ih.trace_ptr, host.trace_ptr)
    assert not np.array_equal(ih.span_id, host.span_id)
    for t in range(0, host.n_traces, 997):
        a, b = int(host.trace_ptr[t]), int(host.trace_ptr[t + 1])
        assert sorted(ih.span_id[a:b].tolist()) == sorted(host.span_id[a:b].tolist())
    assert_table_equal(ctx.edge_aggregate(intra), native.edge_aggregate(ih))


@pytest.mark.slow
def test_large_interleaved_conservation(ctx):
    """2^23 SN traces (~72 M spans) interleaved in 4096-trace windows: the
    grouped edge table equals the table of the original grouped set (span
    ids are unique, so the table does not depend on in-trace order)."""
    dev = ctx.generate(anomod.SynthSpec("SN", seed=20251103, p_orphan_ppm=500), 1 << 23)
    want = ctx.edge_aggregate(dev)
    inter = ctx.shuffle(dev, seed=1, window_traces=4096)
    dev.free()
    got = ctx.edge_aggregate(inter)
    for k in ("count", "errors", "sum_us", "min_us", "max_us", "hist"):
        np.testing.assert_array_equal(getattr(got, k), getattr(want, k), err_msg=k)
    g = ctx.group(inter)
    assert g.n_traces == 1 << 23 and g.n_spans == inter.n_spans


@pytest.mark.slow
def test_full_size_ungrouped_equals_grouped(ctx):
    """The bench's ungrouped workload at its full size (BASELINE config 3 on
    one GPU: 2^27 SN traces, 1.15e9 spans, the spans of every 4096
    consecutive traces interleaved): the table the two-level scatter + join
    path computes equals, bit for bit, the grouped set's table — a
    size-independent property where the oracle cannot follow (unique ids, so
    the table does not depend on in-trace order); the path is the join."""
    dev = ctx.generate(anomod.SynthSpec("SN", seed=20251103, p_orphan_ppm=100), 1 << 27)
    want = ctx.edge_aggregate(dev, with_hist=True)
    inter = ctx.shuffle(dev, seed=20251105, window_traces=4096)
    dev.free()
    got = ctx.edge_aggregate(inter, with_hist=True)
    assert ctx.group_info()["path"] == "join"
    inter.free()
    for k in ("count", "errors", "sum_us", "min_us", "max_us", "hist", "p50_us", "p99_us"):
        np.testing.assert_array_equal(getattr(got, k), getattr(want, k), err_msg=k)
    assert int(got.count.sum()) == int(want.count.sum()) > 10**9


@pytest.fixture
def env_knob(monkeypatch):
    """Set a libanomod environment knob for one test (read on every call)."""
    return monkeypatch.setenv


@pytest.mark.parametrize("path,avg", [("lsd", None), ("bucket", "64"), ("bucket", "1024"),
                                      ("pipe", "1024"), ("pipe", "64")])
def test_group_paths_agree(ctx, env_knob, path, avg):
    """The LSD path (ANOMOD_GROUP_PATH=lsd) and the bucket path at the
    smallest / largest mean bucket size (ANOMOD_BUCKET_AVG: one or two
    scatter levels, most buckets in the small or the large per-bucket
    kernel), also with the persistent pipelined bucket kernel
    (ANOMOD_BK_PIPE=1), give the oracle's grouping."""
    if path == "lsd":
        env_knob("ANOMOD_GROUP_PATH", "lsd")
    else:
        env_knob("ANOMOD_BUCKET_AVG", avg)
    if path == "pipe":
        env_knob("ANOMOD_BK_PIPE", "1")
    rng = np.random.default_rng(77)
    sp = _with_trace_hashes(_random_spanset(rng, 12, 60000, 40, dup=0.02), rng)
    big = _with_trace_hashes(_random_spanset(rng, 12, 4, 1500, dup=0.02), rng)
    flat = _interleave(anomod.SpanSet.concat([sp, big]), rng, "time")
    g = ctx.group(ctx.upload_ungrouped(flat))
    _assert_grouped_equal(g.download(), _oracle_grouped(flat))


def test_group_bucket_overflow(ctx):
    """Traces of 1000-5000 spans overfill their buckets (small per-bucket
    kernel: 2048 spans) and take the large kernel (8192 spans); a bucket
    beyond that makes the call retry with finer buckets, and one holding a
    single 9 000- / 12 000- / 20 000-span trace is copied in arrival order.
    Same grouping every way."""
    rng = np.random.default_rng(78)
    sp = _with_trace_hashes(_random_spanset(rng, 12, 20000, 16, dup=0.02), rng)
    for lens in (rng.integers(1000, 5000, 6), np.r_[12000, rng.integers(1000, 5000, 3)],
                 np.r_[20000, 9000]):
        big = _with_trace_hashes(_random_spanset(rng, 12, 0, 0, dup=0.02, lens=lens), rng)
        flat = _interleave(anomod.SpanSet.concat([sp, big]), rng, "random")
        g = ctx.group(ctx.upload_ungrouped(flat))
        _assert_grouped_equal(g.download(), _oracle_grouped(flat))
        assert ctx.group_info()["path"] == "bucket"


def test_group_huge_buckets(ctx):
    """Traces whose keys share their top 40 bits stay in one bucket however
    fine the split: three long ones (11 000 spans) are ranked by the huge-
    bucket walk; 2100 four-span traces in one bucket (more distinct keys than
    that walk holds) send the call to the LSD path.  Same grouping."""
    rng = np.random.default_rng(79)
    sp = _with_trace_hashes(_random_spanset(rng, 12, 5000, 16, dup=0.02), rng)
    for lens, path in (([4000, 4000, 3000], "bucket"), ([4] * 2100, "lsd")):
        base = rng.integers(0, 2**64, 1, dtype=np.uint64)[0] & np.uint64(0xFFFFFFFFFF000000)
        low = rng.choice(2**24, len(lens), replace=False).astype(np.uint64)
        keys = (base | low).astype(np.uint64)
        big = _with_trace_hashes(_random_spanset(rng, 12, 0, 0, dup=0.02, lens=lens), rng,
                                 _unmix64(keys))
        flat = _interleave(anomod.SpanSet.concat([sp, big]), rng, "random")
        g = ctx.group(ctx.upload_ungrouped(flat))
        _assert_grouped_equal(g.download(), _oracle_grouped(flat))
        assert ctx.group_info()["path"] == path


@pytest.mark.parametrize("avg", [None, "64"])
def test_group_pair_key_collisions(ctx, env_knob, avg):
    """The buckets sort 8-B pairs that carry 32 key bits below level A's;
    traces whose keys agree in all those bits (here: in the top 48) land in
    one run of equal pair keys, interleaved by arrival.  The bucket kernel
    sees the gathered records' full keys differ and re-ranks the bucket by
    (full key, arrival): the oracle's grouping, with one level (default) and
    two (ANOMOD_BUCKET_AVG=64)."""
    if avg:
        env_knob("ANOMOD_BUCKET_AVG", avg)
    rng = np.random.default_rng(80)
    sp = _with_trace_hashes(_random_spanset(rng, 12, 30000, 16, dup=0.02), rng)
    k1 = rng.integers(0, 2**64, 500, dtype=np.uint64)
    k2 = (k1 & np.uint64(0xFFFFFFFFFFFF0000)) | rng.integers(0, 2**16, 500, dtype=np.uint64)
    keep = k2 != k1
    keys = np.concatenate([k1[keep], k2[keep]])
    coll = _with_trace_hashes(_random_spanset(rng, 12, 0, 0, dup=0.02,
                                              lens=rng.integers(1, 30, keys.shape[0])),
                              rng, _unmix64(keys))
    flat = _interleave(anomod.SpanSet.concat([sp, coll]), rng, "time")
    g = ctx.group(ctx.upload_ungrouped(flat))
    _assert_grouped_equal(g.download(), _oracle_grouped(flat))
    assert ctx.group_info()["path"] == "bucket"
    assert ctx.group_info()["levels"] == (2 if avg else 1)


@pytest.mark.parametrize("join", ["1", "0"])
@pytest.mark.parametrize("S,max_len,form", [(12, 24, None), (46, 60, None), (20, 40, None),
                                            (12, 24, "pair"), (100, 30, None)])
def test_ungrouped_fused_equals_unfused(ctx, env_knob, monkeypatch, S, max_len, form, join):
    """anomod_edge_aggregate_ungrouped's fused path (the default: the buckets
    write one edge record per span, the table is taken from those records)
    against the unfused one (ANOMOD_UNGROUPED_FUSED=0: grouped columns, then
    the chunk walk) and the oracle: SN / TrainTicket
    widths (direct, wide, slot stats), wide latencies (a compact-form run that
    learns the set's form), duplicate ids, orphans, interleaved arrival.  join
    "1": the buckets' LDS hash join on (trace, id) (the fused default); "0":
    the sorting bucket kernel's in-trace scan."""
    env_knob("ANOMOD_FUSED_JOIN", join)
    if form:
        env_knob("ANOMOD_HIST_FORM", form)
    rng = np.random.default_rng(S * 3 + max_len)
    sp = _with_trace_hashes(_random_spanset(rng, S, 40000, max_len, dup=0.03,
                                            wide_dur=S == 20), rng)
    flat = _interleave(sp, rng, "time")
    ref = native.edge_aggregate(_oracle_grouped(flat))
    dev = ctx.upload_ungrouped(flat)
    monkeypatch.setenv("ANOMOD_UNGROUPED_FUSED", "1")
    fused = ctx.edge_aggregate(dev)
    assert ctx.group_info()["path"] == ("join" if join == "1" else "fused-sort")
    assert_table_equal(fused, ref)
    monkeypatch.setenv("ANOMOD_UNGROUPED_FUSED", "0")
    assert_table_equal(ctx.edge_aggregate(dev), ref)
    if form is None:  # learned from the compact run (wide latencies: far too many keys)
        assert dev.hints[1] in ((1,) if S == 20 else (0, 1))
    assert_table_equal(ctx.edge_aggregate(dev), ref)  # again, with the learned form
    dev.free()


def test_ungrouped_fused_long_traces_fall_back(ctx, monkeypatch):
    """Buckets of several traces of thousands of spans (beyond the large
    bucket kernel) leave the fused path for the unfused one; the table is
    the oracle's either way."""
    rng = np.random.default_rng(90)
    sp = _with_trace_hashes(_random_spanset(rng, 12, 5000, 16, dup=0.02), rng)
    base = rng.integers(0, 2**64, 1, dtype=np.uint64)[0] & np.uint64(0xFFFFFFFFFF000000)
    low = rng.choice(2**24, 3, replace=False).astype(np.uint64)
    big = _with_trace_hashes(_random_spanset(rng, 12, 0, 0, dup=0.02, lens=[4000, 4000, 3000]),
                             rng, _unmix64((base | low).astype(np.uint64)))
    flat = _interleave(anomod.SpanSet.concat([sp, big]), rng, "random")
    dev = ctx.upload_ungrouped(flat)
    monkeypatch.setenv("ANOMOD_UNGROUPED_FUSED", "1")
    assert_table_equal(ctx.edge_aggregate(dev), native.edge_aggregate(_oracle_grouped(flat)))


def test_ungrouped_join_shared_ids_and_big_buckets(ctx):
    """The join path's edge cases, against the oracle on the stably grouped
    spans: forty traces in ONE bucket (mixed keys sharing their top 40 bits)
    whose span ids and parent ids are identical — the (trace, id) join must
    tell them apart by the trace hash, and each trace's duplicate ids resolve
    to its own first match — and three 900-span traces in one bucket (2 700
    spans: over the join kernel's 2 048, so the sorting large kernel's edge
    form takes it), beside ordinary random traces."""
    rng = np.random.default_rng(77)
    S = 12

    def same_ids(k, L):
        sid = rng.integers(1, 2**63, L, dtype=np.uint64)
        sid[5] = sid[2]  # a repeated id inside the trace: the first match wins
        pid = np.zeros(L, np.uint64)
        pid[1:] = sid[(rng.random(L - 1) * np.arange(1, L)).astype(np.int64)]
        pid[7] = np.uint64(12345)  # an orphan reference
        ptr = np.arange(k + 1, dtype=np.uint64) * np.uint64(L)
        n = k * L
        return anomod.SpanSet([f"svc{i:03d}" for i in range(S)], ptr, np.zeros(n, np.uint64),
                              np.tile(sid, k), np.tile(pid, k),
                              rng.integers(0, S, n).astype(np.uint16),
                              (rng.random(n) < 0.1).astype(np.uint16),
                              rng.integers(50, 5000, n).astype(np.uint32))

    def one_bucket(sp):
        base = rng.integers(0, 2**64, 1, dtype=np.uint64)[0] & np.uint64(0xFFFFFFFFFF000000)
        low = rng.choice(2**24, sp.n_traces, replace=False).astype(np.uint64)
        return _with_trace_hashes(sp, rng, _unmix64((base | low).astype(np.uint64)))

    shared = one_bucket(same_ids(40, 20))
    big = one_bucket(_random_spanset(rng, S, 0, 0, dup=0.02, lens=[900, 900, 900]))
    rest = _with_trace_hashes(_random_spanset(rng, S, 20000, 16, dup=0.02), rng)
    flat = _interleave(anomod.SpanSet.concat([rest, shared, big]), rng, "random")
    dev = ctx.upload_ungrouped(flat)
    got = ctx.edge_aggregate(dev)
    assert ctx.group_info()["path"] == "join"
    assert_table_equal(got, native.edge_aggregate(_oracle_grouped(flat)))
    dev.free()


@pytest.mark.parametrize("pack,stable_b,recb", [("1", "0", "0"), ("0", "0", "0"), ("1", "1", "0"),
                                                ("1", "0", "1"), ("0", "0", "1")])
@pytest.mark.parametrize("S,max_len,dup", [(12, 24, 0.05), (46, 60, 0.02)])
def test_ungrouped_join_two_levels(ctx, env_knob, S, max_len, dup, pack, stable_b, recb):
    """The join path through BOTH scatter levels (ANOMOD_BUCKET_AVG=64 makes a
    ~1 M-span set use T >= 12 bucket bits): level B's non-stable scatter
    (LDS-atomic ranks, the default for the join) with repeated (trace, id)
    resolved by level-A position, against the stable scatter; the packed key
    word (service in the bucket's shared key bits) against the separate
    service array; buckets over 2 048 spans in the big join kernel; the r06
    form whose level B moves the records too (ANOMOD_JOIN_RECB=1: the join
    reads them contiguously).  Every table equals the oracle's on the stably
    grouped spans."""
    env_knob("ANOMOD_BUCKET_AVG", "64")
    env_knob("ANOMOD_JOIN_PACK", pack)
    env_knob("ANOMOD_BK_STABLE_B", stable_b)
    env_knob("ANOMOD_JOIN_RECB", recb)
    rng = np.random.default_rng(S * 7 + int(dup * 100))
    parts = [_random_spanset(rng, S, 60000, max_len, dup=dup)]
    # a few traces of 1 000-3 000 spans: buckets over 2 048 spans (big kernel)
    parts.append(_random_spanset(rng, S, 0, 0, dup=dup, lens=[3000, 1500, 1000, 2500]))
    sp = _with_trace_hashes(anomod.SpanSet.concat(parts), rng)
    flat = _interleave(sp, rng, "time")
    ref = native.edge_aggregate(_oracle_grouped(flat))
    dev = ctx.upload_ungrouped(flat)
    for _ in range(2):
        got = ctx.edge_aggregate(dev)
        info = ctx.group_info()
        assert info["path"] == "join" and info["levels"] == 2 and info["bits"] >= 12, info
        assert_table_equal(got, ref)
    dev.free()


@pytest.mark.parametrize("recb", ["0", "1"])
def test_ungrouped_join_duplicates_across_level_b_tiles(ctx, env_knob, recb):
    """Repeated (trace, id) pairs whose copies are far apart in arrival order
    (other traces' spans between them, so they sit in different level-B tiles
    and land in a bucket in any order once level B is not stable): the
    parent of every child is its trace's FIRST span with that id — the copies
    carry different services, so a wrong pick changes the edge table."""
    env_knob("ANOMOD_BUCKET_AVG", "64")
    env_knob("ANOMOD_JOIN_RECB", recb)
    rng = np.random.default_rng(4242)
    S, nt, L = 12, 30000, 12
    sp = _random_spanset(rng, S, nt, 0, dup=0.0, lens=np.full(nt, L))
    sid = sp.span_id.reshape(nt, L)
    pid = sp.parent_span_id.reshape(nt, L)
    sid[:, 6] = sid[:, 1]  # the id of span 1 again at span 6 ...
    pid[:, 7:] = sid[:, 1:2]  # ... and spans 7.. reference it
    svc = sp.svc.reshape(nt, L)
    svc[:, 1] = 3
    svc[:, 6] = 9  # first match -> service 3, a wrong pick -> 9
    sp = _with_trace_hashes(sp, rng)
    flat = _interleave(sp, rng, "random")
    ref = native.edge_aggregate(_oracle_grouped(flat))
    dev = ctx.upload_ungrouped(flat)
    assert_table_equal(ctx.edge_aggregate(dev), ref)
    assert ctx.group_info()["levels"] == 2
    dev.free()


def test_reserve_grouping_then_aggregate(ctx):
    """anomod_ctx_reserve_grouping sizes the workspace ahead of the first
    call (the join path's part, then both record buffers for a grouping into
    columns); aggregations and groupings after it equal the oracle, and a
    reservation smaller than the workspace is a no-op."""
    rng = np.random.default_rng(31)
    sp = _with_trace_hashes(_random_spanset(rng, 12, 20000, 24, dup=0.02), rng)
    flat = _interleave(sp, rng, "time")
    ref = native.edge_aggregate(_oracle_grouped(flat))
    with anomod.Context(0) as c:
        dev = c.upload_ungrouped(flat)  # reserves the join path's workspace
        h = c.host_ms()
        assert h["group_alloc"][1] == 1
        c.reserve_grouping(flat.n_spans // 2)  # smaller: nothing allocated
        assert c.host_ms()["group_alloc"][1] == 1
        assert_table_equal(c.edge_aggregate(dev), ref)
        assert c.host_ms()["group_alloc"][1] == 1  # the call allocated nothing
        g = c.group(dev)  # grouping into columns: the second record buffer now
        assert c.host_ms()["group_alloc"][1] == 2
        assert_table_equal(c.edge_aggregate(g), ref)
        g.free()
        dev.free()

