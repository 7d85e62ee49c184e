"""Traces longer than a wave chunk (> 256 spans), up to 2*10^5 spans in one
trace, in shuffled in-trace order.  The chunk walk of the edge and
trace-structure kernels lists such traces, and a workgroup-per-trace pass
resolves them (csrc/edge_agg.hip edge_big_kernel, csrc/trace_struct.hip
ts_big_kernel) through LDS hash windows over the trace's ids.

Checker: the C oracle (ordered scans, O(L^2) per trace) up to a few thousand
spans, with duplicated ids and cycles; beyond that the vectorised unique-id
restatement in oracle/spec.py, itself pinned to the C oracle here on CPU."""
import numpy as np
import pytest

import anomod
from oracle import native, spec

TS_FIELDS = ("parent_pos", "depth", "n_children", "span_flags", "n_roots", "svc_mask")
EDGE_FIELDS = ("count", "errors", "sum_us", "min_us", "max_us", "hist")


def _tree_trace(rng, L, orphan=0.01, chain=0.0):
    """One trace of L spans: a random tree (each span's parent an earlier span,
    a `chain` fraction of them the immediately preceding one, so the tree
    holds long paths), a few orphan references, then shuffled in-trace."""
    sid = rng.choice(np.iinfo(np.int64).max, size=L, replace=False).astype(np.uint64) + np.uint64(1)
    pos = np.arange(L)
    par = (rng.random(L) * np.maximum(pos, 1)).astype(np.int64)
    ch = rng.random(L) < chain
    par[ch] = np.maximum(pos[ch] - 1, 0)
    pid = np.where(pos > 0, sid[par], np.uint64(0))
    orph = (pos > 0) & (rng.random(L) < orphan)
    pid[orph] = rng.integers(1, 2**63, int(orph.sum()), dtype=np.uint64) | np.uint64(1 << 63)
    perm = rng.permutation(L)
    return sid[perm], pid[perm]


def _set(rng, S, lens, **kw):
    sids, pids = [], []
    for L in lens:
        s, p = _tree_trace(rng, int(L), **kw)
        sids.append(s)
        pids.append(p)
    ptr = np.zeros(len(lens) + 1, np.uint64)
    np.cumsum(lens, out=ptr[1:])
    n = int(ptr[-1])
    sid = np.concatenate(sids) if sids else np.zeros(0, np.uint64)
    pid = np.concatenate(pids) if pids else np.zeros(0, np.uint64)
    svc = rng.integers(0, S, n).astype(np.uint16)
    flg = (rng.random(n) < 0.1).astype(np.uint16)
    dur = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    dur[rng.random(n) < 0.8] %= 30000
    return anomod.SpanSet([f"s{i:03d}" for i in range(S)], ptr, sid.copy(), sid, pid, svc, flg,
                          dur)


def _mixed_lens(rng, big):
    lens = list(rng.integers(0, 40, 400)) + list(big) + list(rng.integers(0, 30, 300))
    rng.shuffle(lens)
    return lens


# ------------------------------------------------------------------ CPU pins
def test_unique_id_restatement_matches_c_oracle():
    rng = np.random.default_rng(11)
    sp = _set(rng, 9, _mixed_lens(rng, [300, 1200, 2500]), chain=0.3)
    ref = native.edge_aggregate(sp)
    got = spec.unique_id_edge_table(sp, 9)
    for k in EDGE_FIELDS:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    ref = native.trace_structure(sp)
    got = spec.unique_id_trace_structure(sp, 9)
    for k in TS_FIELDS:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    # a parent cycle (no root reached) -> depth 0, as the C oracle
    sp2 = anomod.SpanSet(["a"], np.array([0, 3], np.uint64), np.zeros(3, np.uint64),
                         np.array([5, 6, 7], np.uint64), np.array([6, 5, 0], np.uint64),
                         np.zeros(3, np.uint16), np.zeros(3, np.uint16), np.ones(3, np.uint32))
    got = spec.unique_id_trace_structure(sp2, 1)
    ref = native.trace_structure(sp2)
    for k in TS_FIELDS:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


# ------------------------------------------------------------------ GPU parity
@pytest.mark.gpu
def test_gpu_huge_shuffled_traces_edge_table(ctx):
    rng = np.random.default_rng(21)
    S = 20
    sp = _set(rng, S, _mixed_lens(rng, [200_000, 70_000, 5000, 4097, 257]), chain=0.2)
    got = ctx.edge_aggregate(sp)
    ref = spec.unique_id_edge_table(sp, S)
    for k in ("count", "errors", "sum_us", "min_us", "max_us"):
        np.testing.assert_array_equal(getattr(got, k), ref[k], err_msg=k)
    np.testing.assert_array_equal(got.hist, ref["hist"])
    # exact per-edge quantiles take the same long-trace pass (key mode)
    q, _ = ctx.edge_quantiles_exact(sp, (50, 99))
    e = ref["edge"]
    d = sp.dur_us.astype(np.int64)
    for edge in np.unique(e)[:50]:
        x = np.sort(d[e == edge])
        assert q[edge, 0] == x[len(x) * 50 // 100] and q[edge, 1] == x[len(x) * 99 // 100]


@pytest.mark.gpu
def test_gpu_huge_shuffled_traces_structure(ctx):
    rng = np.random.default_rng(22)
    S = 70  # two service words
    sp = _set(rng, S, _mixed_lens(rng, [150_000, 30_000, 4096, 300]), chain=0.995)
    got = ctx.trace_structure(sp)
    ref = spec.unique_id_trace_structure(sp, S)
    for k in TS_FIELDS:
        np.testing.assert_array_equal(getattr(got, k), ref[k], err_msg=k)
    assert got.depth.max() > 300  # long parent chains went through pointer jumping


@pytest.mark.gpu
def test_gpu_long_traces_duplicates_and_cycles(ctx):
    """Duplicated ids (longest-path relaxation), forward references (cycles)
    and id 0 in traces of 257..6000 spans: C oracle, bit-exact."""
    rng = np.random.default_rng(23)
    S = 12
    lens = _mixed_lens(rng, [6000, 2049, 700, 257])
    sp = _set(rng, S, lens, chain=0.3)
    ptr = sp.trace_ptr.astype(np.int64)
    n = sp.n_spans
    dup = rng.random(n) < 0.03
    src = rng.integers(0, n, n)
    t_of = np.repeat(np.arange(len(lens)), np.diff(ptr))
    same = t_of[src] == t_of
    sp.span_id[dup & same] = sp.span_id[src[dup & same]]
    fwd = rng.random(n) < 0.01
    sp.parent_span_id[fwd & same] = sp.span_id[src[fwd & same]]
    sp.span_id[rng.random(n) < 0.002] = 0
    ref = native.trace_structure(sp)
    got = ctx.trace_structure(sp)
    for k in TS_FIELDS:
        np.testing.assert_array_equal(getattr(got, k), ref[k], err_msg=k)
    ref = native.edge_aggregate(sp)
    got = ctx.edge_aggregate(sp)
    for k in ("count", "errors", "sum_us", "min_us", "max_us"):
        np.testing.assert_array_equal(getattr(got, k), ref[k], err_msg=k)
    np.testing.assert_array_equal(got.hist, ref["hist"])


@pytest.mark.gpu
def test_gpu_long_topology_device_generation_and_parity(ctx):
    """SynthSpec LONG (SN services, traces of 16..4000 spans, 30 % of the spans
    past the wave path): device generation == host generation, edge table and
    trace structure == the C oracle."""
    spec = anomod.SynthSpec("LONG", seed=4, p_orphan_ppm=2000)
    n = 3000
    dev = ctx.generate(spec, n)
    host = anomod.synth_generate_host(spec, n)
    got = dev.download()
    for k in ("trace_ptr", "span_id", "parent_span_id", "svc", "flags", "dur_us"):
        np.testing.assert_array_equal(getattr(got, k), getattr(host, k), err_msg=k)
    assert np.diff(host.trace_ptr).max() > 1000
    ref = native.edge_aggregate(host)
    t = ctx.edge_aggregate(dev)
    for k in ("count", "errors", "sum_us", "min_us", "max_us"):
        np.testing.assert_array_equal(getattr(t, k), ref[k], err_msg=k)
    np.testing.assert_array_equal(t.hist, ref["hist"])
    ref = native.trace_structure(host)
    ts = ctx.trace_structure(dev)
    for k in TS_FIELDS:
        np.testing.assert_array_equal(getattr(ts, k), ref[k], err_msg=k)

