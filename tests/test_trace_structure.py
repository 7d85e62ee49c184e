"""Trace structure: the C oracle against the reference's
own _build_span_records outputs (tests/golden/skywalking_small.json and
skywalking_dups.json — duplicated node ids with different parents, where the
BFS keeps a node's deepest visit — written by tests/golden/gen/make_goldens.py),
then the HIP kernel against the oracle
(bit-exact) on the goldens and on random span sets with duplicate ids, parent
cycles, orphans and traces longer than a wave chunk."""
import json

import numpy as np
import pytest

import anomod
from anomod import decode
from oracle import native

NO_PARENT = 0xFFFFFFFF
FIELDS = ("parent_pos", "depth", "n_children", "span_flags", "n_roots", "svc_mask")


GOLDENS = ("skywalking_small.json", "skywalking_dups.json")


def _golden_set(golden, name="skywalking_small.json"):
    g = json.loads((golden / name).read_text())
    kept = [(spans, exp) for spans, exp in zip(g["inputs"], g["expected"]) if exp["node_ids"]]
    sp = anomod.decode_skywalking_raw([s for s, _ in kept])
    return sp, kept


def _check_against_reference(sp, kept, ts):
    ptr = sp.trace_ptr.astype(np.int64)
    assert len(kept) == sp.n_traces
    for t, (spans, exp) in enumerate(kept):
        a, b = ptr[t], ptr[t + 1]
        nodes, _, _ = decode.skywalking_parents(spans)
        assert nodes == exp["node_ids"]
        pp = ts["parent_pos"][a:b]
        # the reference's parent_node_id is the raw reference; it names a span
        # of the trace exactly when parent_pos is set
        for k, (p, ref_parent) in enumerate(zip(pp, exp["parent_node_ids"])):
            if p != NO_PARENT:
                assert nodes[p] == ref_parent
            else:
                assert ref_parent is None or ref_parent not in nodes
        assert ts["depth"][a:b].tolist() == exp["depths"]
        assert ts["n_children"][a:b].tolist() == [len(c) for c in exp["children"]]
        fl = ts["span_flags"][a:b]
        roots = [nodes[k] for k in range(b - a) if fl[k] == (1 | 2)]
        assert roots == exp["roots"]
        assert int(ts["n_roots"][t]) == len(exp["roots"])
        mask = ts["svc_mask"][t] if ts["svc_mask"].ndim == 2 else ts["svc_mask"][t:t + 1]
        names = [s for i, s in enumerate(sp.services) if (int(mask[i // 64]) >> (i % 64)) & 1]
        assert names == exp["services_involved"]


@pytest.mark.parametrize("name", GOLDENS)
def test_oracle_matches_reference_build_span_records(golden, name):
    sp, kept = _golden_set(golden, name)
    _check_against_reference(sp, kept, native.trace_structure(sp))


def _random_set(rng, S, n_traces, max_len, dup=0.05, cycle=0.02):
    lens = rng.integers(0, max_len + 1, n_traces)
    ptr = np.zeros(n_traces + 1, np.uint64)
    np.cumsum(lens, out=ptr[1:])
    n = int(ptr[-1])
    sid = rng.integers(1, 2**63, n, dtype=np.uint64)
    pid = np.zeros(n, np.uint64)
    t_of = np.repeat(np.arange(n_traces), lens)
    starts = ptr[:-1].astype(np.int64)[t_of]
    ends = ptr[1:].astype(np.int64)[t_of]
    pos = np.arange(n) - starts
    has = pos > 0
    pick = starts + (rng.random(n) * np.maximum(pos, 1)).astype(np.int64)
    pid[has] = sid[pick[has]]
    fwd = has & (rng.random(n) < cycle)  # references to later spans: cycles possible
    later = starts + (rng.random(n) * (ends - starts)).astype(np.int64)
    pid[fwd] = sid[np.minimum(later[fwd], n - 1)]
    orph = has & (rng.random(n) < 0.05)
    pid[orph] = rng.integers(1, 2**63, int(orph.sum()), dtype=np.uint64)
    d = has & (rng.random(n) < dup)
    sid[d] = sid[pick[d]]
    svc = rng.integers(0, S, n).astype(np.uint16)
    return anomod.SpanSet([f"s{i:03d}" for i in range(S)], ptr, sid.copy(), sid, pid, svc,
                          np.zeros(n, np.uint16), np.ones(n, np.uint32))


def test_oracle_self_consistency():
    rng = np.random.default_rng(5)
    sp = _random_set(rng, 7, 300, 25)
    ts = native.trace_structure(sp)
    ptr = sp.trace_ptr.astype(np.int64)
    for t in range(sp.n_traces):
        a, b = ptr[t], ptr[t + 1]
        fl = ts["span_flags"][a:b]
        assert int(ts["n_roots"][t]) == int((fl == 3).sum())
        roots = ts["parent_pos"][a:b] == NO_PARENT
        assert ((fl & 1) == 1).tolist() == roots.tolist()
        # a root node is re-visited deeper when a duplicate of it has a
        # resolving parent (the BFS keeps the last visit), so only traces
        # with unique ids pin root depths to 0
        if len(set(sp.span_id[a:b].tolist())) == b - a:
            assert (ts["depth"][a:b][roots] == 0).all()


# ---------------------------------------------------------------- GPU parity
def _gpu_equal(ctx, sp):
    got = ctx.trace_structure(sp)
    ref = native.trace_structure(sp)
    for k in FIELDS:
        np.testing.assert_array_equal(getattr(got, k), ref[k], err_msg=k)
    return got


@pytest.mark.gpu
@pytest.mark.parametrize("name", GOLDENS)
def test_gpu_matches_reference_goldens(ctx, golden, name):
    sp, kept = _golden_set(golden, name)
    got = _gpu_equal(ctx, sp)
    _check_against_reference(sp, kept, {k: getattr(got, k) for k in FIELDS})


@pytest.mark.gpu
@pytest.mark.parametrize("S,n_traces,max_len", [(3, 3000, 12), (12, 20000, 30), (46, 4000, 60),
                                                (100, 2000, 40)])
def test_gpu_random_sets_bit_exact(ctx, S, n_traces, max_len):
    _gpu_equal(ctx, _random_set(np.random.default_rng(S + n_traces), S, n_traces, max_len))


@pytest.mark.gpu
@pytest.mark.parametrize("n_traces", [1, 513, (1 << 19) + 3])
def test_gpu_dynamic_tail_segments_bit_exact(ctx, n_traces):
    """The second half of the traces goes out in 512-trace segments from a
    device counter (re-zeroed per call): each trace resolved exactly once."""
    sp = _random_set(np.random.default_rng(n_traces), 12, n_traces, 6)
    _gpu_equal(ctx, sp)
    _gpu_equal(ctx, sp)


@pytest.mark.gpu
def test_gpu_big_traces_and_empty(ctx):
    rng = np.random.default_rng(9)
    parts = [_random_set(rng, 12, 40, 10), _random_set(rng, 12, 2, 900),
             _random_set(rng, 12, 100, 20), _random_set(rng, 12, 1, 257)]
    sp = anomod.SpanSet.concat(parts)
    assert np.diff(sp.trace_ptr).max() > 256
    _gpu_equal(ctx, sp)
    empty = anomod.SpanSet(["a"], np.zeros(3, np.uint64), *(np.zeros(0, t) for t in (
        np.uint64, np.uint64, np.uint64, np.uint16, np.uint16, np.uint32)))
    got = ctx.trace_structure(empty)
    assert got.n_roots.tolist() == [0, 0] and got.depth.size == 0


@pytest.mark.gpu
def test_gpu_synthetic_sn_device_resident(ctx):
    spec = anomod.SynthSpec("SN", seed=3, p_orphan_ppm=2000)
    dev = ctx.generate(spec, 30000)
    got = ctx.trace_structure(dev)
    ref = native.trace_structure(dev.download())
    for k in FIELDS:
        np.testing.assert_array_equal(getattr(got, k), ref[k], err_msg=k)
    # SN templates: one root per trace unless the generator dropped a parent
    assert (got.n_roots >= 1).all()


@pytest.mark.gpu
def test_gpu_scratch_reuse_across_sizes():
    """r06: the outputs and the long-trace scratch live in the context's
    scratch slots and are reused, not freed: a larger set, then a smaller one
    (the slot is larger than the call needs; nothing of the previous call may
    show), then one with long traces (the long-trace slot grows), then the
    first again — every call equal to the oracle."""
    rng = np.random.default_rng(21)
    big = _random_set(rng, 12, 30000, 30)
    small = _random_set(rng, 5, 700, 12)
    longs = anomod.SpanSet.concat([_random_set(rng, 12, 50, 20), _random_set(rng, 12, 3, 1200)])
    with anomod.Context(0) as c:
        for sp in (big, small, longs, small, big):
            _gpu_equal(c, sp)
