"""Product decoders (anomod.decode) against the reference goldens."""
import csv
import io
import json

import numpy as np

import anomod
from anomod import decode
from oracle import spec


def _csv_rows(path):
    with open(path, newline="") as fh:
        return list(csv.DictReader(fh))


def test_decode_jaeger_matches_reference_csv(golden):
    doc = json.loads((golden / "jaeger_small.json").read_text())
    ref = _csv_rows(golden / "jaeger_small.csv")
    sp = anomod.decode_jaeger(doc)
    assert sp.n_spans == len(ref)
    assert sp.n_traces == len(doc["data"])
    tix = sp.trace_of_span()
    for i, row in enumerate(ref):
        assert sp.trace_ids[tix[i]] == row["trace_id"]
        assert int(sp.span_id[i]) == decode.jaeger_id(row["span_id"])
        assert int(sp.parent_span_id[i]) == decode.jaeger_id(row["parent_span_id"])
        assert sp.services[sp.svc[i]] == row["service"]
        assert int(sp.dur_us[i]) == int(row["duration_us"])
        tags = json.loads(row["tags"])
        err = tags.get("error") is True or str(tags.get("http.status_code", "")).isdigit() and \
            int(tags["http.status_code"]) >= 500
        assert bool(sp.flags[i] & anomod.FLAG_ERROR) == bool(err)
    assert sp.services == sorted(set(r["service"] for r in ref))


def test_decode_jaeger_empty(golden):
    sp = anomod.decode_jaeger({"data": []})
    assert sp.n_spans == 0 and sp.n_traces == 0
    assert _csv_rows(golden / "jaeger_empty.csv") == []


def test_jaeger_ids():
    assert decode.jaeger_id("") == 0
    assert decode.jaeger_id("00000000000000ff") == 255
    assert decode.jaeger_id("0000000000000000") != 0
    assert decode.jaeger_id("not-hex") >> 63 == 1
    assert decode.jaeger_id("123") == 0x123


def _expected_parent_index(nodes, parents):
    first = {}
    for i, n in enumerate(nodes):
        first.setdefault(n, i)
    return [None if p is None else first.get(p, -1) for p in parents]


def _check_sw(sp, expected):
    for t, exp in enumerate([e for e in expected if e["node_ids"]]):
        a, b = int(sp.trace_ptr[t]), int(sp.trace_ptr[t + 1])
        assert b - a == len(exp["node_ids"])
        want = _expected_parent_index(exp["node_ids"], exp["parent_node_ids"])
        sid = sp.span_id[a:b].tolist()
        for k, w in enumerate(want):
            pid = int(sp.parent_span_id[a + k])
            if w is None:
                assert pid == 0
            elif w == -1:
                assert pid not in sid and pid != 0
            else:
                assert sid.index(pid) == w
        assert [sp.services[c] for c in sp.svc[a:b]] == [s or "" for s in exp["service_code"]]
        assert (sp.dur_us[a:b] == np.asarray(exp["duration_ms"]) * 1000).all()
        assert (sp.flags[a:b].astype(bool) == np.asarray(exp["is_error"])).all()
        # roots of the reference == spans whose parent is absent or unresolved
        roots = [exp["node_ids"][k] for k, w in enumerate(want) if w is None or w == -1]
        assert set(roots) == set(exp["roots"])


def test_decode_skywalking_raw_matches_reference(golden):
    g = json.loads((golden / "skywalking_small.json").read_text())
    sp = anomod.decode_skywalking_raw(g["inputs"])
    _check_sw(sp, g["expected"])


def test_decode_skywalking_payload_matches_reference(golden):
    g = json.loads((golden / "skywalking_small.json").read_text())
    sp = anomod.decode_skywalking_payload(g["payload"])
    _check_sw(sp, g["expected"])


def test_skywalking_parents_match_oracle(golden):
    g = json.loads((golden / "skywalking_small.json").read_text())
    for spans in g["inputs"]:
        nodes, parents, _ = anomod.skywalking_parents(spans)
        recs, _ = spec.build_span_records(spans)
        assert nodes == [r["node_id"] for r in recs]
        assert parents == [r["parent_node_id"] for r in recs]


def test_decoders_agree_with_oracle_edge_table(golden):
    from oracle import native
    doc = json.loads((golden / "jaeger_small.json").read_text())
    sp = anomod.decode_jaeger(doc)
    tab = native.edge_aggregate(sp)
    py = spec.edge_table_py(sp, sp.n_services)
    assert tab["count"].tolist() == py["count"]
    assert int(tab["count"].sum()) == sp.n_spans


def test_merge_jaeger_dumps_sorted_dedup():
    d1 = {"data": [{"traceID": "b", "k": 1}, {"traceID": "a", "k": 1}]}
    d2 = {"data": [{"traceID": "c", "k": 2}, {"traceID": "a", "k": 2}]}
    m = anomod.merge_jaeger_dumps([d1, {"data": []}, d2])
    assert [t["traceID"] for t in m["data"]] == ["a", "b", "c"]
    assert [t["k"] for t in m["data"]] == [1, 1, 2]  # first occurrence kept


def test_metric_long_csv_dedup_and_nan():
    buf = io.StringIO()
    w = csv.writer(buf)
    w.writerow(["metric_name", "timestamp", "datetime", "value", "instance", "pod"])
    for rep in range(2):  # duplicated query (metric_collector.py key_metrics repeats)
        for t in (0, 15, 30):
            w.writerow(["process_open_fds", t, "x", "" if t == 15 else str(10 + t + rep), "i1", ""])
            w.writerow(["up", t, "x", "1", "i1", "ts-order-service-abc"])
    buf.seek(0)
    mm = anomod.decode_metric_long_csv(buf)
    assert mm.S == 2 and mm.T == 3
    assert mm.series[0] == ("process_open_fds", (("instance", "i1"),))
    col = mm.X[:, 0]
    assert col[0] == 10 and np.isnan(col[1]) and col[2] == 40
    padded = mm.pad_to_multiple(2)
    assert padded.T == 4 and np.isnan(padded.X[3]).all()


def _prom_expected(results: dict):
    """Series of the SN metric directory derived from the stubbed Prometheus
    answers themselves: key (file stem, label string as
    fetch_prometheus_metrics.py:51 renders it) -> {epoch: value}."""
    exp = {}
    for stem, result in results.items():
        for r in result:
            labels = ",".join(f'{k}="{v}"' for k, v in r.get("metric", {}).items())
            exp[(stem, (("metric", labels),))] = {float(t): float(v) for t, v in r["values"]}
    return exp


def test_prometheus_dir_matches_reference_csvs(golden, monkeypatch):
    """decode_prometheus_csv_dir on the CSVs the reference's
    fetch_prometheus_metrics() + to_csv wrote (tests/golden/prom_dir, TZ=UTC)
    is column-equal to the query answers that produced them."""
    import time
    monkeypatch.setenv("TZ", "UTC")
    time.tzset()
    try:
        results = json.loads((golden / "prom_results.json").read_text())
        files = sorted(p.stem for p in (golden / "prom_dir").glob("*.csv"))
        # the no-data query writes no file (fetch_prometheus_metrics.py:101-102)
        assert files == sorted(s for s, r in results.items() if r)
        mm = anomod.decode_prometheus_csv_dir(golden / "prom_dir")
        exp = _prom_expected(results)
        assert sorted(mm.series) == sorted(exp) and list(mm.series) == sorted(mm.series)
        want_ts = sorted({t for d in exp.values() for t in d})
        np.testing.assert_allclose(mm.timestamps, want_ts, rtol=0, atol=1e-6)
        col_of = {t: i for i, t in enumerate(want_ts)}
        for j, key in enumerate(mm.series):
            want = np.full(mm.T, np.nan, np.float32)
            for t, v in exp[key].items():
                want[col_of[t]] = np.float32(v)
            np.testing.assert_array_equal(mm.X[:, j], want)
        # specials survive the CSV round trip
        assert np.isposinf(mm.X).any() and np.isneginf(mm.X).any() and np.isnan(mm.X).any()
        assert any(k[1][0][1] == "" for k in mm.series)  # empty label set
    finally:
        monkeypatch.undo()
        time.tzset()
