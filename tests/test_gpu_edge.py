"""GPU parity: HIP edge aggregation (libanomod) vs the CPU oracle, bit-exact."""
import json

import numpy as np
import pytest

import anomod
from oracle import native, spec

pytestmark = pytest.mark.gpu

FIELDS = ("count", "errors", "sum_us", "min_us", "max_us")


def assert_table_equal(gpu: anomod.EdgeTable, ref: dict):
    for k in FIELDS:
        np.testing.assert_array_equal(getattr(gpu, k), ref[k], err_msg=k)
    if gpu.hist is not None:
        np.testing.assert_array_equal(gpu.hist, ref["hist"], err_msg="hist")
    ref = native.finalize(ref)
    np.testing.assert_array_equal(gpu.p50_us, ref["p50_us"])  # NaN == NaN here
    np.testing.assert_array_equal(gpu.p99_us, ref["p99_us"])


def _random_spanset(rng, S, n_traces, max_len, orphan=0.05, dup=0.0, wide_dur=True,
                    lo_alias=False, lens=None):
    if lens is None:
        lens = rng.integers(0, max_len + 1, n_traces)
    lens = np.asarray(lens, np.int64)
    n_traces = lens.shape[0]
    ptr = np.zeros(n_traces + 1, np.uint64)
    np.cumsum(lens, out=ptr[1:])
    n = int(ptr[-1])
    sid = rng.integers(1, 2**63, n, dtype=np.uint64)
    if lo_alias:  # ids that share their low 32-bit word with other ids of the trace
        sid = (sid & np.uint64(0x7FFFFFFF00000000)) | rng.integers(1, 4, n, dtype=np.uint64)
    pid = np.zeros(n, np.uint64)
    t_of = np.repeat(np.arange(n_traces), lens)
    starts = ptr[:-1].astype(np.int64)[t_of]
    pos = np.arange(n) - starts
    has_parent = pos > 0
    pick = starts + (rng.random(n) * np.maximum(pos, 1)).astype(np.int64)
    pid[has_parent] = sid[pick[has_parent]]
    orph = has_parent & (rng.random(n) < orphan)
    pid[orph] = rng.integers(1, 2**63, int(orph.sum()), dtype=np.uint64)
    if lo_alias:  # orphan references whose low word matches ids of the trace
        pid[orph] = (pid[orph] & np.uint64(0x7FFFFFFF00000000)) | rng.integers(
            1, 4, int(orph.sum()), dtype=np.uint64)
    if dup:
        d = has_parent & (rng.random(n) < dup)
        sid[d] = sid[pick[d]]  # duplicate span ids inside a trace
    svc = rng.integers(0, S, n).astype(np.uint16)
    flg = (rng.random(n) < 0.1).astype(np.uint16)
    if wide_dur:
        dur = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        dur[rng.random(n) < 0.7] %= 20000
    else:
        dur = rng.integers(50, 5000, n).astype(np.uint32)
    return anomod.SpanSet([f"svc{i:03d}" for i in range(S)], ptr, sid.copy(), sid, pid, svc, flg,
                          dur)


def test_native_library_is_loaded(ctx):
    assert anomod.LIB_PATH.exists()
    assert anomod.device_count() >= 1


@pytest.mark.parametrize("S,n_traces,max_len", [
    (1, 100, 5), (3, 2000, 12), (12, 20000, 24), (20, 5000, 30),  # LDS-stat variants
    (46, 5000, 60),   # TrainTicket width: compact 22-bit keys, wide per-edge stats
    (47, 3000, 60),   # E = 2303: the widest table with wide stats
    (48, 3000, 60),   # E = 2400: slot-hashed stats
    (100, 2000, 40),  # compact keys, slot-hashed stats
])
def test_random_sets_bit_exact(ctx, S, n_traces, max_len):
    rng = np.random.default_rng(S * 1000 + n_traces)
    sp = _random_spanset(rng, S, n_traces, max_len, dup=0.02)
    assert_table_equal(ctx.edge_aggregate(sp), native.edge_aggregate(sp))


@pytest.mark.parametrize("n_traces", [1, 511, 513, 16387, (1 << 20) + 1])
def test_dynamic_tail_segments_bit_exact(ctx, n_traces):
    """The kernel splits the first 3/4 of the traces statically over its waves
    and hands the last 1/4 out in 512-trace segments from a device counter:
    every trace is counted exactly once at counts around those boundaries
    (fewer traces than waves, one segment and a bit, many segments)."""
    rng = np.random.default_rng(n_traces)
    sp = _random_spanset(rng, 12, n_traces, 6, dup=0.01)
    assert_table_equal(ctx.edge_aggregate(sp), native.edge_aggregate(sp))
    again = ctx.edge_aggregate(sp)  # the counter is re-zeroed per launch
    assert_table_equal(again, native.edge_aggregate(sp))


@pytest.mark.parametrize("S,max_len", [(12, 40), (46, 60)])
def test_low_word_aliases(ctx, S, max_len):
    """Span ids sharing their low 32-bit word inside a trace: the kernel scans
    low words and must confirm the high word (false candidates, orphans whose
    low word matches, duplicates), incl. traces longer than one chunk."""
    rng = np.random.default_rng(S + 99)
    parts = [_random_spanset(rng, S, 3000, max_len, dup=0.05, lo_alias=True),
             _random_spanset(rng, S, 4, 700, lo_alias=True)]
    sp = anomod.SpanSet.concat(parts)
    assert_table_equal(ctx.edge_aggregate(sp), native.edge_aggregate(sp))


@pytest.mark.parametrize("dup", [0.0, 0.05])
def test_low_word_aliases_long_windows(ctx, dup):
    """The long-trace resolve keys its slots by the low id word and confirms
    the high word staged by position (r06): traces of 300-5 000 spans (packed
    windows and traces over one 2 048-id window) whose ids share low words
    three ways, orphans whose low word matches, repeated ids (the first
    position must keep the slot).  Equal to the oracle."""
    rng = np.random.default_rng(777 + int(dup * 100))
    parts = [_random_spanset(rng, 12, 0, 0, dup=dup, lo_alias=True,
                             lens=list(rng.integers(300, 2049, 12)) + [2049, 3000, 5000])]
    parts.append(_random_spanset(rng, 12, 2000, 40, dup=dup, lo_alias=True))
    sp = anomod.SpanSet.concat(parts)
    assert_table_equal(ctx.edge_aggregate(sp), native.edge_aggregate(sp))
    q, _ = ctx.edge_quantiles_exact(sp, (50, 99))
    np.testing.assert_array_equal(q, native.exact_quantiles(sp, (50, 99)))


@pytest.mark.parametrize("S,long_set", [(46, False), (12, True)])
def test_low_word_aliases_unique_ids(ctx, monkeypatch, S, long_set):
    """Unique ids (so the split-word scan runs: TrainTicket width, and the
    long-trace instantiation for a set holding a trace over 256 spans) whose
    low 32-bit words collide inside the trace: a low-word candidate whose
    high word differs must not count — the scan falls back to the exact one.
    Collector order and shuffled inside the traces.  Equal to the oracle."""
    if long_set:
        monkeypatch.setenv("ANOMOD_HIST_FORM", "compact")
    rng = np.random.default_rng(500 + S)
    parts = [_random_spanset(rng, S, 3000, 60, lo_alias=True)]
    if long_set:
        parts.append(_random_spanset(rng, S, 0, 0, lo_alias=True,
                                     lens=rng.integers(100, 257, 300)))
        parts.append(_random_spanset(rng, S, 0, 0, lo_alias=True, lens=[300]))
    sp = anomod.SpanSet.concat(parts)
    assert sp.check_unique_ids()
    dev = ctx.upload(sp)
    assert_table_equal(ctx.edge_aggregate(dev), native.edge_aggregate(sp))
    shuf = ctx.shuffle(dev, seed=11, window_traces=0)
    assert_table_equal(ctx.edge_aggregate(shuf), native.edge_aggregate(shuf.download()))
    shuf.free()
    dev.free()


@pytest.mark.parametrize("S,lens", [(46, (30, 200)), (46, (1, 25)), (12, (30, 200))])
def test_fingerprint_collisions(ctx, S, lens):
    """Ids crafted so that EVERY id of the set — orphan references included —
    shares lo ^ hi (the value any fingerprint, bucket or hash scheme over the
    ids would key on; DESIGN §7 logs the ones measured), with duplicated ids:
    the first-match rule has to be decided on the full 64-bit ids."""
    rng = np.random.default_rng(S * 31 + lens[1])
    sp = _random_spanset(rng, S, 3000, 0, dup=0.05,
                         lens=rng.integers(lens[0], lens[1] + 1, 3000))

    def one_fp(x):
        hi = x >> np.uint64(32)
        return (hi << np.uint64(32)) | (hi ^ np.uint64(0x5A5A5A5A))

    sp.span_id[:] = one_fp(sp.span_id)
    nz = sp.parent_span_id != 0
    sp.parent_span_id[nz] = one_fp(sp.parent_span_id[nz])
    assert_table_equal(ctx.edge_aggregate(sp), native.edge_aggregate(sp))


def test_big_traces(ctx):
    rng = np.random.default_rng(7)
    parts = [_random_spanset(rng, 12, 50, 10), _random_spanset(rng, 12, 3, 3000),
             _random_spanset(rng, 12, 200, 20), _random_spanset(rng, 12, 1, 257)]
    sp = anomod.SpanSet.concat(parts)
    assert np.diff(sp.trace_ptr).max() > 256
    assert_table_equal(ctx.edge_aggregate(sp), native.edge_aggregate(sp))


def test_empty_and_degenerate(ctx):
    svcs = ["a", "b"]
    empty = anomod.SpanSet(svcs, np.zeros(1, np.uint64), *(np.zeros(0, t) for t in
                           (np.uint64, np.uint64, np.uint64, np.uint16, np.uint16, np.uint32)))
    t = ctx.edge_aggregate(empty)
    assert t.count.sum() == 0 and np.isnan(t.p50_us).all()
    assert (t.min_us == 0xFFFFFFFF).all()
    # traces with zero spans between real ones, self-parent, parent == 0
    sp = anomod.SpanSet(svcs, np.array([0, 0, 3, 3, 4], np.uint64),
                        np.zeros(4, np.uint64), np.array([5, 6, 7, 9], np.uint64),
                        np.array([0, 5, 6, 9], np.uint64), np.array([0, 1, 1, 0], np.uint16),
                        np.array([1, 0, 0, 0], np.uint16),
                        np.array([0, 2**32 - 1, 64, 7], np.uint32))
    assert_table_equal(ctx.edge_aggregate(sp), native.edge_aggregate(sp))


def test_counter_wrap_and_table_saturation(ctx):
    # one (edge, bin) hit millions of times: exercises the packed-count wrap
    n = 3_000_000
    ptr = np.arange(0, n + 1, 2, dtype=np.uint64)
    sid = np.arange(1, n + 1, dtype=np.uint64)
    pid = np.where(np.arange(n) % 2 == 1, sid - 1, 0).astype(np.uint64)
    sp = anomod.SpanSet(["x", "y"], ptr, sid, sid, pid, (np.arange(n) % 2).astype(np.uint16),
                        np.zeros(n, np.uint16), np.full(n, 1234, np.uint32))
    assert_table_equal(ctx.edge_aggregate(sp), native.edge_aggregate(sp))
    # every bin of many edges: more distinct keys than LDS slots
    rng = np.random.default_rng(11)
    sp = _random_spanset(rng, 16, 60000, 30)
    sp.dur_us[:] = rng.integers(0, 2**32, sp.n_spans, dtype=np.uint64).astype(np.uint32)
    assert_table_equal(ctx.edge_aggregate(sp), native.edge_aggregate(sp))


def test_device_generation_matches_host(ctx):
    for topo, n in (("SN", 50000), ("TT", 5000)):
        spec = anomod.SynthSpec(topo, seed=99, p_orphan_ppm=3000,
                                fault_service=3)
        dev = ctx.generate(spec, n)
        host = anomod.synth_generate_host(spec, n)
        got = dev.download()
        for k in ("trace_ptr", "trace_hash", "span_id", "parent_span_id", "svc", "flags",
                  "dur_us"):
            np.testing.assert_array_equal(getattr(got, k), getattr(host, k), err_msg=k)
        assert_table_equal(ctx.edge_aggregate(dev), native.edge_aggregate(host))


def test_tt_device_set_1e7_spans_bit_exact(ctx):
    """TrainTicket width at ~1.0e7 spans (compact histogram + wide stats),
    generated in HBM, against the C oracle on the host-generated twin."""
    spec = anomod.SynthSpec("TT", seed=5, p_orphan_ppm=500, fault_service=7, fault_latency_mult=9)
    n = 440_000
    dev = ctx.generate(spec, n)
    assert dev.n_spans >= 10_000_000
    host = anomod.synth_generate_host(spec, n)
    assert_table_equal(ctx.edge_aggregate(dev), native.edge_aggregate(host))


def test_jaeger_golden_edge_table(ctx, golden):
    doc = json.loads((golden / "jaeger_small.json").read_text())
    sp = anomod.decode_jaeger(doc)
    assert_table_equal(ctx.edge_aggregate(sp), native.edge_aggregate(sp))


def test_skywalking_golden_edge_table(ctx, golden):
    g = json.loads((golden / "skywalking_small.json").read_text())
    sp = anomod.decode_skywalking_raw(g["inputs"])
    assert_table_equal(ctx.edge_aggregate(sp), native.edge_aggregate(sp))


def test_shards_sum_to_whole(ctx):
    sp = anomod.synth_generate_host(anomod.SynthSpec("SN", seed=5, p_orphan_ppm=1000), 40000)
    whole = ctx.edge_aggregate(sp)
    parts = [ctx.edge_aggregate(sp.shard(3, r)) for r in range(3)]
    np.testing.assert_array_equal(sum(p.count for p in parts), whole.count)
    np.testing.assert_array_equal(sum(p.hist for p in parts), whole.hist)
    np.testing.assert_array_equal(np.minimum.reduce([p.min_us for p in parts]), whole.min_us)
    np.testing.assert_array_equal(np.maximum.reduce([p.max_us for p in parts]), whole.max_us)


@pytest.mark.slow
def test_large_synthetic_full_parity(ctx):
    """~72 M spans generated in HBM: full oracle parity + conservation of the
    first call (auto form) and of the second — the instantiation bench.py's
    headline times — histogram and quantiles included (the nearest-rank rule
    of monitor_http_responses.py:183-190 on the merged histogram)."""
    spec = anomod.SynthSpec("SN", seed=20251103, p_orphan_ppm=500)
    dev = ctx.generate(spec, 1 << 23)
    # (the generator declares collector order; the histogram form is not known)
    assert dev.unique_ids and dev.hints == (1, -1)
    t1 = ctx.edge_aggregate(dev)  # first call: the auto form (pair + resume hand-off)
    # the call the bench times runs edge_agg_kernel<lds_hist,lds_stats,unique>
    # (the bidirectional scan of a collector-order unique-id set, pair form)
    assert dev.hints == (1, 0)
    t2 = ctx.edge_aggregate(dev)
    assert int(t1.count.sum()) == dev.n_spans
    np.testing.assert_array_equal(t1.hist.sum(axis=1), t1.count)
    host = dev.download()
    ref = native.edge_aggregate(host)
    assert_table_equal(t1, ref)
    assert_table_equal(t2, ref)  # hist, p50 / p99 included


@pytest.mark.parametrize("cap", [1000, 4096])
def test_multi_launch_split_bit_exact(ctx, monkeypatch, cap):
    """Span sets above the per-launch span bound (2^32 - 1: a workgroup's u32
    LDS counters must not wrap) run as several launches over whole trace ranges;
    ANOMOD_MAX_LAUNCH_SPANS lowers the bound so the split runs here: cuts
    inside runs of short traces, a trace longer than the bound alone, empty
    traces at the cuts."""
    rng = np.random.default_rng(cap)
    parts = [_random_spanset(rng, 12, 3000, 12, dup=0.01), _random_spanset(rng, 12, 2, 5000),
             _random_spanset(rng, 12, 700, 3), _random_spanset(rng, 12, 1, 1)]
    sp = anomod.SpanSet.concat(parts)
    ref = native.edge_aggregate(sp)
    monkeypatch.setenv("ANOMOD_MAX_LAUNCH_SPANS", str(cap))
    assert_table_equal(ctx.edge_aggregate(sp), ref)
    monkeypatch.delenv("ANOMOD_MAX_LAUNCH_SPANS")
    assert_table_equal(ctx.edge_aggregate(sp), ref)


@pytest.mark.slow
def test_tt_full_size_one_launch_equals_two(ctx, monkeypatch):
    """2^27 TrainTicket traces (3.1e9 spans: above 2^31, below 2^32): one
    launch gives the same table as two launches cut at 2^31 spans."""
    dev = ctx.generate(anomod.SynthSpec("TT", seed=20251103, p_orphan_ppm=100), 1 << 27)
    assert (1 << 31) < dev.n_spans < (1 << 32) - 1
    one = ctx.edge_aggregate(dev)
    monkeypatch.setenv("ANOMOD_MAX_LAUNCH_SPANS", str(1 << 31))
    two = ctx.edge_aggregate(dev)
    monkeypatch.delenv("ANOMOD_MAX_LAUNCH_SPANS")
    dev.free()
    for k in FIELDS + ("hist", "p50_us", "p99_us"):
        np.testing.assert_array_equal(getattr(one, k), getattr(two, k), err_msg=k)
    assert int(one.count.sum()) > (1 << 31)


@pytest.mark.parametrize("S,n_traces,max_len", [(12, 20000, 24), (46, 4000, 60), (3, 1, 3000)])
def test_exact_quantiles_match_sorted_latencies(ctx, S, n_traces, max_len):
    """§8a a11 cross-check mode: exact per-edge order statistics on the GPU
    (edge keys from the aggregation walk + one radix sort) == numpy sort of
    each edge's latencies; the histogram quantile sits within its bin."""
    rng = np.random.default_rng(S + n_traces)
    sp = _random_spanset(rng, S, n_traces, max_len, dup=0.02)
    q = (0, 50, 57, 95, 99)  # 57: int(c * 0.57) != (c * 57) // 100 for c = 100
    got, cnt = ctx.edge_quantiles_exact(sp, q)
    want = native.exact_quantiles(sp, q)
    np.testing.assert_array_equal(got, want)
    tab = native.finalize(native.edge_aggregate(sp))
    np.testing.assert_array_equal(cnt, tab["count"])
    ok = cnt > 0
    for k, qq in ((1, "p50_us"), (4, "p99_us")):  # histogram midpoint vs exact: same bin
        ex = got[ok, k].astype(np.uint32)
        b = [spec.hist_bounds(spec.hist_bin(int(v))) for v in ex]
        np.testing.assert_array_equal(tab[qq][ok], [0.5 * (lo + hi) for lo, hi in b])


def test_exact_quantiles_scratch_reuse_across_sizes():
    """r06: the exact quantiles keep their workspace in a context scratch
    slot: a large set, a small one (stale keys past its end must not count),
    a larger one with long traces (the slot grows), the small one again."""
    rng = np.random.default_rng(23)
    big = _random_spanset(rng, 12, 20000, 24, dup=0.02)
    small = _random_spanset(rng, 7, 300, 9)
    longs = anomod.SpanSet.concat([_random_spanset(rng, 12, 30000, 24),
                                   _random_spanset(rng, 12, 0, 0, lens=[700, 2500])])
    with anomod.Context(0) as c:
        for sp in (big, small, longs, small):
            got, cnt = c.edge_quantiles_exact(sp, (50, 99))
            np.testing.assert_array_equal(got, native.exact_quantiles(sp, (50, 99)))
            assert int(cnt.sum()) == sp.n_spans


def test_exact_quantiles_first_call_on_new_context():
    """The exact quantiles as a fresh context's first call on a unique-id set
    whose scan order is not known yet: the order probe needs the pinned
    read-back the aggregation would otherwise have allocated (ADVICE r05:
    it wrote through a null staging pointer)."""
    with anomod.Context(0) as maker:
        gen = maker.generate(anomod.SynthSpec("SN", seed=7, p_orphan_ppm=100), 4096)
        host = gen.download()
        gen.free()
    assert host.unique_ids
    host.scan_order = -1  # order unknown: the exact quantiles' probe runs
    with anomod.Context(0) as fresh:
        dev = fresh.upload(host)
        assert dev.hints[0] == -1
        got, cnt = fresh.edge_quantiles_exact(dev, (50, 99))
        assert dev.hints[0] in (0, 1)
        dev.free()
    want = native.exact_quantiles(host, (50, 99))
    np.testing.assert_array_equal(got, want)
    assert int(cnt.sum()) == host.n_spans


@pytest.mark.parametrize("form", ["pair", "compact", "auto"])
@pytest.mark.parametrize("S", [14, 46])
def test_histogram_forms(ctx, monkeypatch, form, S):
    """Both LDS histogram forms of the SN-width (E <= 512, direct stats) and
    TrainTicket-width (E <= 2304, wide stats) kernels, and the form-unknown
    first aggregation (pair form; saturated workgroups hand their traces to a
    compact resume launch), give the oracle's table bit for bit
    (ANOMOD_HIST_FORM forces each)."""
    monkeypatch.setenv("ANOMOD_HIST_FORM", form)
    rng = np.random.default_rng(61 + S)
    sp = _random_spanset(rng, S, 30000, 40, dup=0.01)
    assert_table_equal(ctx.edge_aggregate(sp), native.edge_aggregate(sp))
    dev = ctx.generate(anomod.SynthSpec("LONG", seed=8, p_orphan_ppm=500), 2000)
    ref = native.edge_aggregate(dev.download())
    assert_table_equal(ctx.edge_aggregate(dev), ref)
    dev.free()


def test_pair_table_overflow_switches_form(ctx):
    """A device set touching far more (edge, bin) keys per workgroup than the
    pair table's 8 Ki slots (random call trees over 20 services, latencies
    over the whole u32 range) saturates it on the first aggregation — whose
    stopped workgroups hand their traces to the compact resume launch — and
    later aggregations take the compact form at once.  Every result, the
    first included, equals the oracle's."""
    rng = np.random.default_rng(62)
    sp = _random_spanset(rng, 20, 700_000, 40)
    ref = native.edge_aggregate(sp)
    dev = ctx.upload(sp)
    assert not dev.hist_compact and dev.hints == (-1, -1)
    for _ in range(3):
        assert_table_equal(ctx.edge_aggregate(dev), ref)
        assert dev.hist_compact and dev.hints[1] == 1
    dev.free()


def test_first_aggregation_has_no_cliff(ctx):
    """The first aggregation of a fresh LONG set (random call trees over every
    SN service pair: ~15 k (edge, bin) keys per workgroup, twice what the pair
    table holds) costs about what the later ones do (r03: 140x, the probe
    chains and contended HBM counters of a saturated pair table), equals the
    oracle, and a host SpanSet keeps the learned form across uploads."""
    dev = ctx.generate(anomod.SynthSpec("LONG", seed=9), 1 << 20)
    host = dev.download()
    assert host.hist_form == -1
    ref = native.edge_aggregate(host)
    ms = []
    for _ in range(3):
        assert_table_equal(ctx.edge_aggregate(dev), ref)
        ms.append(ctx.stage_ms(0))
    assert dev.hints[1] == 1
    assert ms[0] <= 3.0 * max(ms[1:]) + 0.5, ms
    dev.free()
    assert_table_equal(ctx.edge_aggregate(host), ref)  # uploaded per call
    assert host.hist_form == 1 and host.scan_order == 1


@pytest.mark.parametrize("cap", [3000, 50000])
def test_first_aggregation_multi_launch(ctx, monkeypatch, cap):
    """The saturation hand-off per launch of a multi-launch split (every
    launch's stopped workgroups resume in compact form before the next
    launch re-zeroes the counters)."""
    rng = np.random.default_rng(cap + 1)
    sp = anomod.SpanSet.concat([_random_spanset(rng, 20, 100_000, 40),
                                _random_spanset(rng, 20, 2, 4000)])
    ref = native.edge_aggregate(sp)
    monkeypatch.setenv("ANOMOD_MAX_LAUNCH_SPANS", str(cap))
    monkeypatch.setenv("ANOMOD_HIST_FORM", "auto")
    assert_table_equal(ctx.edge_aggregate(sp), ref)


@pytest.mark.parametrize("S,max_len", [(12, 24), (46, 80), (5, 256)])
def test_unique_id_bidirectional_scan(ctx, monkeypatch, S, max_len):
    """Sets whose span ids are unique within every trace (checked exactly on
    the host) take the bidirectional parent scan; the table equals the
    oracle's and the forward-scan build's (ANOMOD_UNIQUE_SCAN=0), parents
    before and after their children (in-trace shuffle), orphans included."""
    rng = np.random.default_rng(S * 7 + max_len)
    sp = _random_spanset(rng, S, 20000, max_len, orphan=0.03)
    assert sp.check_unique_ids()
    ref = native.edge_aggregate(sp)
    dev = ctx.upload(sp)
    assert dev.unique_ids and dev.scan_order == -1
    shuf = ctx.shuffle(dev, seed=5, window_traces=0)  # parents anywhere in the trace
    assert shuf.unique_ids
    host = shuf.download()
    ref2 = native.edge_aggregate(host)
    # the bidirectional scan forced (=1), the set's own choice, the forward scan
    for scan in ("1", None, "0"):
        if scan is None:
            monkeypatch.delenv("ANOMOD_UNIQUE_SCAN", raising=False)
        else:
            monkeypatch.setenv("ANOMOD_UNIQUE_SCAN", scan)
        assert_table_equal(ctx.edge_aggregate(dev), ref)
        assert_table_equal(ctx.edge_aggregate(shuf), ref2)
    assert shuf.scan_order == 0  # probed: shuffled inside the traces
    shuf.free()
    dev.free()


def test_scan_order_probe(ctx):
    """Generated sets are declared in collector order; shuffling inside the
    traces makes the probe pick the forward scan; the table is the same."""
    gen = ctx.generate(anomod.SynthSpec("TT", seed=9), 20000)
    assert gen.scan_order == 1
    shuf = ctx.shuffle(gen, seed=3, window_traces=0)
    assert shuf.scan_order == -1
    t1, t2 = ctx.edge_aggregate(gen), ctx.edge_aggregate(shuf)
    assert shuf.scan_order == 0
    for k in FIELDS + ("hist",):
        np.testing.assert_array_equal(getattr(t1, k), getattr(t2, k), err_msg=k)


def test_duplicate_ids_are_not_declared_unique(ctx):
    rng = np.random.default_rng(70)
    sp = _random_spanset(rng, 12, 5000, 30, dup=0.05)
    assert not sp.check_unique_ids()
    dev = ctx.upload(sp)
    assert not dev.unique_ids
    assert_table_equal(ctx.edge_aggregate(dev), native.edge_aggregate(sp))
    gen = ctx.generate(anomod.SynthSpec("SN", seed=3), 1000)
    assert gen.unique_ids and gen.download().check_unique_ids()


@pytest.mark.parametrize("alias", [False, True])
def test_long_set_wide_scan(ctx, monkeypatch, capfd, alias):
    """Sets holding a trace longer than a chunk take the long-trace kernel
    instantiation (the wide split-word scan, compact form).
    Traces of 49..256 spans with random ancestors, unique ids per trace;
    alias: every trace reuses the same id values, so a chunk holds equal ids
    of different traces (the lookup keeps to the span's own trace).  Orphans,
    roots, a 300-span trace for the long-trace pass.  Equal to the oracle,
    and the instantiation is the one that ran (random ancestors are not
    collector order, so the bidirectional scans are forced on)."""
    monkeypatch.setenv("ANOMOD_HIST_FORM", "compact")
    monkeypatch.setenv("ANOMOD_UNIQUE_SCAN", "1")
    monkeypatch.setenv("ANOMOD_LOG_KERNEL", "1")
    rng = np.random.default_rng(71 + alias)
    lens = np.r_[rng.integers(49, 257, 600), rng.integers(1, 40, 400), [300]]
    rng.shuffle(lens)
    sp = _random_spanset(rng, 12, 0, 0, lens=lens)
    if alias:  # ids 1..L inside each trace, parents remapped to them
        sp = _alias_ids(sp)
    assert sp.check_unique_ids()
    ref = native.edge_aggregate(sp)
    dev = ctx.upload(sp)
    capfd.readouterr()
    for _ in range(2):
        assert_table_equal(ctx.edge_aggregate(dev), ref)
    assert "wide_scan" in capfd.readouterr().err
    dev.free()


@pytest.mark.parametrize("self_ref", [0.0, 0.1])
def test_long_set_hash_chains(ctx, monkeypatch, capfd, self_ref):
    """The long-trace instantiation on ids crafted so that every id of the
    set — orphan references included — has the same m = (lo ^ hi *
    0x85EBCA77) * 0x9E3779B1 (mod 2^32): the key of the per-chunk id table
    measured in r06 (not kept), under which a chunk's ids fill
    one probe chain with equal tags.  Whatever keys a lookup uses, such ids
    must be told apart by the full 64-bit id and the span's trace.  Random
    ancestors, spans that reference their own id, traces of 1..256 spans and
    a 300-span trace.  Equal to the oracle."""
    monkeypatch.setenv("ANOMOD_HIST_FORM", "compact")
    monkeypatch.setenv("ANOMOD_UNIQUE_SCAN", "1")
    monkeypatch.setenv("ANOMOD_LOG_KERNEL", "1")
    rng = np.random.default_rng(4242 + int(self_ref * 10))
    lens = np.r_[rng.integers(100, 257, 300), rng.integers(1, 30, 200), [300]]
    rng.shuffle(lens)
    sp = _random_spanset(rng, 12, 0, 0, lens=lens)
    n = sp.n_spans
    M = 0x13572468

    def same_m(hi):  # the lo word that gives every hi the same m
        return (np.uint64(M) ^ ((hi * np.uint64(0x85EBCA77)) & np.uint64(0xFFFFFFFF)))

    # distinct high words for the ids, other high words for orphan references
    his = rng.permutation(np.arange(1, 2 * n + 1, dtype=np.uint64) * np.uint64(977))
    sid_hi = his[:n]
    remap = dict(zip(sp.span_id.tolist(), (sid_hi << np.uint64(32) | same_m(sid_hi)).tolist()))
    sid = np.array([remap[int(x)] for x in sp.span_id], np.uint64)
    orph_hi = his[n:]
    pid = np.zeros(n, np.uint64)
    for j, p in enumerate(sp.parent_span_id.tolist()):
        if p:
            if p in remap:
                pid[j] = remap[p]
            else:
                h = orph_hi[j]
                pid[j] = (int(h) << 32) | int(same_m(h))
    if self_ref:
        m = rng.random(n) < self_ref
        pid[m] = sid[m]
    sp = anomod.SpanSet(sp.services, sp.trace_ptr, sid.copy(), sid, pid, sp.svc, sp.flags,
                        sp.dur_us)
    assert sp.check_unique_ids()
    ref = native.edge_aggregate(sp)
    dev = ctx.upload(sp)
    capfd.readouterr()
    assert_table_equal(ctx.edge_aggregate(dev), ref)
    assert "wide_scan" in capfd.readouterr().err
    dev.free()


def _alias_ids(sp, self_ref=0.0, rng=None):
    """The same set with ids 1..L inside every trace (parents remapped to
    them, orphan references to ids no trace holds); self_ref: that share of
    the spans reference their own id."""
    ptr = sp.trace_ptr.astype(np.int64)
    sid = np.empty(sp.n_spans, np.uint64)
    remap = {}
    for t in range(sp.n_traces):
        a, b = ptr[t], ptr[t + 1]
        new = np.arange(1, b - a + 1, dtype=np.uint64)
        remap.update(zip(sp.span_id[a:b].tolist(), new.tolist()))
        sid[a:b] = new
    pid = np.array([remap.get(int(p), 10**12 + int(p) % 997) if p else 0
                    for p in sp.parent_span_id], np.uint64)
    if self_ref:
        m = rng.random(sp.n_spans) < self_ref
        pid[m] = sid[m]
    return anomod.SpanSet(sp.services, sp.trace_ptr, sid.copy(), sid, pid, sp.svc, sp.flags,
                          sp.dur_us)


@pytest.mark.parametrize("S", [12, 46])
def test_aliased_ids_in_chunk(ctx, S):
    """Every trace holds ids 1..L, so a wave chunk holds equal ids of
    different traces on both sides of every trace boundary: the scan's
    forward block runs past the trace end and its backward block is clamped
    at the trace start (re-reading the span itself and later ones), and a
    match there must not count.  SN width (mask-built scan) and TrainTicket
    width (select-built scan), collector order and shuffled inside the
    traces, orphans and self references.  Equal to the oracle."""
    rng = np.random.default_rng(300 + S)
    sp = _alias_ids(_random_spanset(rng, S, 6000, 40, orphan=0.05), self_ref=0.01, rng=rng)
    assert sp.check_unique_ids()
    dev = ctx.upload(sp)
    assert_table_equal(ctx.edge_aggregate(dev), native.edge_aggregate(sp))
    shuf = ctx.shuffle(dev, seed=9, window_traces=0)
    assert shuf.unique_ids
    assert_table_equal(ctx.edge_aggregate(shuf), native.edge_aggregate(shuf.download()))
    shuf.free()
    dev.free()


@pytest.mark.parametrize("shuffle", [False, True])
def test_first_call_form_probe(ctx, shuffle):
    """A set's first aggregation (histogram form unknown) runs its first
    ~2^20 spans in the compact form on a few workgroups, reads their slot
    occupancy and runs the rest in the form that says — an ordinary launch,
    no spilling auto form: it costs about what a later call costs, learns
    the pair form for SN spans (collector order or shuffled inside traces)
    and equals the oracle."""
    dev = ctx.generate(anomod.SynthSpec("SN", seed=31, p_orphan_ppm=500), 1 << 22)
    if shuffle:
        d2 = ctx.shuffle(dev, seed=4)
        dev.free()
        dev = d2
    assert dev.hints[1] == -1
    t1 = ctx.edge_aggregate(dev, with_hist=True)
    cold = ctx.stage_ms(0)
    assert dev.hints[1] == 0
    warm = []
    for _ in range(3):
        t2 = ctx.edge_aggregate(dev, with_hist=True)
        warm.append(ctx.stage_ms(0))
    for k in FIELDS + ("hist",):
        np.testing.assert_array_equal(getattr(t1, k), getattr(t2, k))
    assert cold <= 1.25 * min(warm) + 0.25, (cold, warm)
    assert_table_equal(t1, native.edge_aggregate(dev.download()))
    dev.free()
