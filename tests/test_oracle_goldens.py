"""Pin the CPU oracle against golden vectors produced by the reference's own
code (tests/golden/gen/make_goldens.py) and by pandas / networkx."""
import csv
import json
import random

import numpy as np
import pytest

from oracle import native, spec


def _csv_rows(path):
    with open(path, newline="") as fh:
        return list(csv.DictReader(fh))


def test_jaeger_rows_match_reference_csv(golden):
    doc = json.loads((golden / "jaeger_small.json").read_text())
    ref = _csv_rows(golden / "jaeger_small.csv")
    mine = spec.jaeger_rows(doc)
    assert len(mine) == len(ref) > 100
    for a, b in zip(mine, ref):
        assert a["trace_id"] == b["trace_id"]
        assert a["span_id"] == b["span_id"]
        assert a["parent_span_id"] == b["parent_span_id"]
        assert a["service"] == b["service"]
        assert int(a["duration_us"]) == int(b["duration_us"])
        assert json.dumps(a["tags"]) == b["tags"]


def test_jaeger_empty_is_header_only(golden):
    rows = _csv_rows(golden / "jaeger_empty.csv")
    assert rows == []
    header = (golden / "jaeger_empty.csv").read_text().strip().split(",")
    assert header[:4] == ["trace_id", "span_id", "parent_span_id", "service"]
    assert spec.jaeger_rows({"data": []}) == []


def test_build_span_records_match_reference(golden):
    g = json.loads((golden / "skywalking_small.json").read_text())
    for spans, exp in zip(g["inputs"], g["expected"]):
        recs, roots = spec.build_span_records(spans)
        assert [r["node_id"] for r in recs] == exp["node_ids"]
        assert [r["parent_node_id"] for r in recs] == exp["parent_node_ids"]
        assert [r["depth"] for r in recs] == exp["depths"]
        assert [r["children"] for r in recs] == exp["children"]
        assert [r["duration_ms"] for r in recs] == exp["duration_ms"]
        assert [r["is_error"] for r in recs] == exp["is_error"]
        assert roots == exp["roots"]


def test_analyze_trace_patterns_match_reference(golden):
    g = json.loads((golden / "analyze_patterns.json").read_text())
    mine = spec.analyze_trace_patterns(g["traces"])
    ref = g["analysis"]
    for k in ("total_traces", "unique_services", "unique_endpoints", "error_traces",
              "service_call_counts", "endpoint_call_counts"):
        assert mine[k] == ref[k], k
    assert mine["latency_stats"]["count"] == ref["latency_stats"]["count"]
    assert mine["latency_stats"]["min"] == ref["latency_stats"]["min"]
    assert mine["latency_stats"]["max"] == ref["latency_stats"]["max"]
    assert mine["latency_stats"]["avg"] == pytest.approx(ref["latency_stats"]["avg"], rel=1e-15)
    assert mine["time_range"]["earliest"] == ref["time_range"]["earliest"]
    assert mine["time_range"]["latest"] == ref["time_range"]["latest"]


def test_nearest_rank_matches_reference(golden):
    cases = json.loads((golden / "percentiles.json").read_text())
    for c in cases:
        lat = [v for v in c["latencies"] if v > 0]  # monitor_http_responses.py:167-169
        st = c["latency_statistics"]
        if not lat:
            assert st == {}
            continue
        assert spec.nearest_rank(lat, 50) == st["median"]
        assert spec.nearest_rank(lat, 95) == st["p95"]
        assert spec.nearest_rank(lat, 99) == st["p99"]
        # histogram quantile == exact nearest rank when every value is < 64
        small = [v for v in lat if v < 64]
        if small:
            h = np.zeros((1, native.BINS), np.uint64)
            for v in small:
                h[0, native.hist_bin(v)] += 1
            for q in (50, 95, 99):
                assert native.quantiles(h, q)[0] == spec.nearest_rank(small, q)


def test_hist_bin_c_matches_python():
    vals = [0, 1, 31, 32, 63, 64, 65, 127, 128, 129, 255, 256, 1000, 4095, 4096, 65535,
            2**20 + 7, 2**31 - 1, 2**31, 2**32 - 1]
    vals += [random.Random(1).randrange(2**32) for _ in range(2000)]
    for v in vals:
        b = spec.hist_bin(v)
        assert native.hist_bin(v) == b
        lo, hi = spec.hist_bounds(b)
        assert lo <= v <= hi
        assert 0 <= b < native.BINS
    assert spec.hist_bin(2**32 - 1) == native.BINS - 1
    # bins tile the u32 range without gaps
    prev_hi = -1
    for b in range(native.BINS):
        lo, hi = spec.hist_bounds(b)
        assert lo == prev_hi + 1
        prev_hi = hi
    assert prev_hi == 2**32 - 1


def test_ewma_state_matches_pandas(golden):
    g = np.load(golden / "ewma_pandas.npz")
    X, M, V, a = g["X"], g["mean"], g["var"], float(g["alpha"])
    for s in range(X.shape[1]):
        m, v = spec.ewma_state(X[:, s], a)
        ok = ~np.isnan(M[:, s])
        np.testing.assert_allclose(m[ok], M[ok, s], rtol=1e-12, atol=1e-9)
        np.testing.assert_allclose(v[ok], V[ok, s], rtol=1e-9, atol=1e-9)


def test_ewma_native_matches_pandas_windows(golden):
    g = np.load(golden / "ewma_pandas.npz")
    X, M, V, a = g["X"], g["mean"], g["var"], float(g["alpha"])
    W, eps = 60, 1e-12
    ref = spec.window_scores_from_state(X, M, V, W, eps)
    Z = native.ewma_z(X, a, W, eps)
    np.testing.assert_allclose(Z, ref, rtol=1e-5, atol=1e-6)


def test_pagerank_native_matches_networkx(golden):
    g = np.load(golden / "pagerank_networkx.npz")
    x, it = native.pagerank(g["row_ptr"], g["col"], g["w"], g["p"], float(g["alpha"]),
                            iters=1000, tol=1e-12)
    assert it < 1000
    assert np.abs(x - g["x"]).sum() < 1e-7


def _random_spanset(rng, S, n_traces, max_len, orphan=0.05):
    from anomod.spans import SpanSet
    lens = rng.integers(0, max_len + 1, n_traces)
    ptr = np.zeros(n_traces + 1, np.uint64)
    np.cumsum(lens, out=ptr[1:])
    n = int(ptr[-1])
    sid = rng.integers(1, 2**63, n, dtype=np.uint64)
    pid = np.zeros(n, np.uint64)
    for t in range(n_traces):
        a, b = int(ptr[t]), int(ptr[t + 1])
        for i in range(a + 1, b):
            r = rng.random()
            pid[i] = (rng.integers(1, 2**63, dtype=np.uint64) if r < orphan
                      else sid[rng.integers(a, i)])
    svc = rng.integers(0, S, n).astype(np.uint16)
    flg = (rng.random(n) < 0.1).astype(np.uint16)
    dur = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    dur[rng.random(n) < 0.5] %= 5000
    return SpanSet([f"s{i}" for i in range(S)], ptr, sid.copy(), sid, pid, svc, flg, dur)


def test_native_edge_aggregate_matches_python():
    rng = np.random.default_rng(0)
    for S, nt, ml in [(3, 50, 6), (12, 200, 20), (5, 10, 300)]:
        sp = _random_spanset(rng, S, nt, ml)
        tab = native.finalize(native.edge_aggregate(sp))
        py = spec.edge_table_py(sp, S)
        for k in ("count", "errors", "sum_us", "min_us", "max_us"):
            assert tab[k].tolist() == py[k], k
        h = {(int(e), int(b)): int(tab["hist"][e, b]) for e, b in zip(*np.nonzero(tab["hist"]))}
        assert h == py["hist"]
        assert int(tab["count"].sum()) == sp.n_spans


def test_group_by_trace_is_a_stable_grouping():
    """oracle/spec.py group_by_trace (the rule anomod_spans_group follows)
    against a dict-based restatement: traces by mix64(hash), arrival order
    inside a trace."""
    rng = np.random.default_rng(4)
    th = rng.integers(0, 50, 3000).astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    order, tptr = spec.group_by_trace(th)
    groups: dict = {}
    for i, h in enumerate(th.tolist()):
        groups.setdefault(h, []).append(i)
    keys = sorted(groups, key=lambda h: int(spec.mix64([h])[0]))
    want = [i for h in keys for i in groups[h]]
    assert order.tolist() == want
    assert np.diff(tptr).tolist() == [len(groups[h]) for h in keys]
    assert spec.group_by_trace(np.zeros(0, np.uint64))[1].tolist() == [0]
    # mix64 is the SplitMix64 finaliser
    assert int(spec.mix64([1])[0]) == 0x5692161D100B05E5


def test_exact_edge_quantiles_follow_reference_percentiles(golden):
    """oracle exact per-edge order statistics == the reference's own
    generate_summary picks (sorted(x)[len//2], [int(n*0.99)]) on the
    latency lists of tests/golden/percentiles.json, placed on one edge."""
    import anomod
    cases = json.loads((golden / "percentiles.json").read_text())
    checked = 0
    for case in cases:
        lat = [v for v in case["latencies"] if v > 0]
        if not lat or not all(float(v).is_integer() for v in lat):
            continue
        checked += 1
        n = len(lat)
        sp = anomod.SpanSet(["a"], np.array([0, n], np.uint64), np.zeros(n, np.uint64),
                            np.arange(1, n + 1, dtype=np.uint64), np.zeros(n, np.uint64),
                            np.zeros(n, np.uint16), np.zeros(n, np.uint16),
                            np.asarray(lat, np.uint32))
        q = native.exact_quantiles(sp, (50, 95, 99))
        ref = case["latency_statistics"]  # written by the reference's generate_summary
        assert (q[1, 0], q[1, 1], q[1, 2]) == (ref["median"], ref["p95"], ref["p99"])
    assert checked >= 5


def test_exact_rank_is_pythons_int_of_the_product():
    """The exact-mode index is the reference's int(n * q) (Python f64
    product, truncated; monitor_http_responses.py:188-189) for any q_pct, not
    (n * q_pct) // 100 — they differ e.g. at n = 100, q = 0.57."""
    import anomod
    from oracle import native

    sp = anomod.SpanSet(["a"], np.array([0, 100], np.uint64), np.ones(100, np.uint64),
                        np.arange(1, 101, dtype=np.uint64), np.zeros(100, np.uint64),
                        np.zeros(100, np.uint16), np.zeros(100, np.uint16),
                        np.arange(100, dtype=np.uint32)[::-1].copy())
    got = native.exact_quantiles(sp, tuple(range(100)), S=1)
    row = 1 * 1 + 0  # ROOT -> a
    for q in range(100):
        assert got[row, q] == sorted(range(100))[int(100 * (q / 100))]
    assert got[row, 57] == 56 and (100 * 57) // 100 == 57
