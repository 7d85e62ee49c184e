"""Native decoders (csrc/decode.cpp) column-equal to the
Python decoders, which are pinned to the reference's own outputs
(test_decode.py / test_oracle_goldens.py).  Host-only: no GPU needed."""
import json
import random

import numpy as np
import pytest

import anomod
from anomod import _lib as L
from anomod import decode

COLS = ("trace_ptr", "trace_hash", "span_id", "parent_span_id", "svc", "flags", "dur_us")


def _same(a, b):
    assert a.services == b.services
    for k in COLS:
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k), err_msg=k)
    # the native decoder's own per-trace id check == the exact host check
    assert a.unique_ids == b.check_unique_ids()


def test_decoder_unique_ids_flag():
    """anomod_decoded_unique_ids: 1 for a payload whose node ids are unique in
    every trace (a synthetic collector payload), 0 once one trace repeats a
    node id; the same as SpanSet.check_unique_ids on the decoded columns."""
    from anomod import writers

    sp = anomod.synth_generate_host(anomod.SynthSpec("TT", seed=3), 40)
    doc = writers.skywalking_payload(sp, "u")
    got = anomod.decode_native(json.dumps(doc).encode(), "skywalking")
    assert got.unique_ids and got.check_unique_ids()
    doc["traces"][7]["spans"][3]["node_id"] = doc["traces"][7]["spans"][1]["node_id"]
    got = anomod.decode_native(json.dumps(doc).encode(), "skywalking")
    assert not got.unique_ids and not got.check_unique_ids()


def test_hash64_matches_python():
    lib = L.lib()
    rng = random.Random(1)
    for s in ["", "a", "abc", "x" * 31, "y" * 32, "z" * 33, "ü€😀", "7c2fc07fa518f930"] + [
            "".join(rng.choice("0123456789abcdef") for _ in range(rng.randint(1, 80)))
            for _ in range(200)]:
        b = s.encode()
        assert lib.anomod_hash64(b, len(b)) == decode.hash64(s)


def test_jaeger_golden_native_equals_python(golden):
    data = (golden / "jaeger_small.json").read_bytes()
    _same(anomod.decode_native(data, "jaeger"), decode.decode_jaeger(json.loads(data)))


def test_skywalking_payload_native_equals_python(golden):
    g = json.loads((golden / "skywalking_small.json").read_text())
    data = json.dumps(g["payload"]).encode()
    _same(anomod.decode_native(data, "skywalking"), decode.decode_skywalking_payload(g["payload"]))
    data2 = json.dumps(g["payload"], indent=2, ensure_ascii=False).encode()  # collector's format
    _same(anomod.decode_native(data2, "skywalking"),
          decode.decode_skywalking_payload(g["payload"]))


def _messy_jaeger(rng, n_traces=60):
    svcs = ["svc-α", "svc \"q\"", "svc\\b", "plain", "emoji😀"]
    data = []
    for t in range(n_traces):
        procs = {f"p{k}": {"serviceName": rng.choice(svcs)} for k in range(3)}
        spans = []
        ids = [("%016x" % rng.getrandbits(64)) if rng.random() < 0.8 else
               rng.choice(["", "0", "zz-not-hex", "00000000000000000001", "0000000000000000"])
               for _ in range(rng.randint(0, 12))]
        for j, sid in enumerate(ids):
            refs = []
            if j and rng.random() < 0.9:
                refs.append({"refType": rng.choice(["CHILD_OF", "FOLLOWS_FROM"]),
                             "spanID": rng.choice(ids[:j])})
                if rng.random() < 0.3:
                    refs.append({"refType": "CHILD_OF", "spanID": rng.choice(ids)})
            tags = []
            for _ in range(rng.randint(0, 4)):
                k = rng.choice(["error", "http.status_code", "component", "x"])
                v = rng.choice([True, False, "true", "TRUE", "false", 200, 503, "503", " 500 ",
                                "5_03", "499", 503.7, 12.0, "abc", None, -1])
                tags.append({"key": k, "type": "x", "value": v})
            dur = rng.choice([0, 1, 123, 2**32 + 5, -4, 17.9, "88", "x", None])
            sp = {"traceID": "t", "spanID": sid, "operationName": "op", "references": refs,
                  "startTime": 1762207158839501 + j, "duration": dur, "tags": tags,
                  "logs": [], "processID": rng.choice(["p0", "p1", "p2", "p9"])}
            if rng.random() < 0.05:
                del sp["references"]
            spans.append(sp)
        data.append({"traceID": rng.choice(["%032x" % rng.getrandbits(128), "", "tr\\u00e9"]),
                     "spans": spans, "processes": procs})
    return {"data": data}


@pytest.mark.parametrize("seed", range(5))
def test_jaeger_messy_native_equals_python(seed):
    doc = _messy_jaeger(random.Random(seed))
    for text in (json.dumps(doc), json.dumps(doc, indent=2, ensure_ascii=False),
                 json.dumps(doc, separators=(",", ":"))):
        _same(anomod.decode_native(text.encode(), "jaeger"), decode.decode_jaeger(json.loads(text)))


def test_service_list_and_errors(golden):
    data = (golden / "jaeger_small.json").read_bytes()
    py = decode.decode_jaeger(json.loads(data))
    fixed = ["zzz-extra"] + py.services
    got = anomod.decode_native(data, "jaeger", fixed)
    assert got.services == fixed
    np.testing.assert_array_equal(got.svc, py.svc + 1)
    with pytest.raises(anomod.AnomodError):
        anomod.decode_native(data, "jaeger", ["only-one"])
    with pytest.raises(anomod.AnomodError):
        anomod.decode_native(b'{"data": [1, 2', "jaeger")
    empty = anomod.decode_native(b'{"data": []}', "jaeger")
    assert empty.n_spans == 0 and empty.n_traces == 0


def test_load_trace_file_dispatch(golden, tmp_path):
    g = json.loads((golden / "skywalking_small.json").read_text())
    p = tmp_path / "x_skywalking_traces_1.json"
    p.write_text(json.dumps(g["payload"], indent=2))
    _same(anomod.load_trace_file(p), decode.decode_skywalking_payload(g["payload"]))
    r = tmp_path / "raw.json"
    r.write_text(json.dumps(g["inputs"]))
    _same(anomod.load_trace_file(r), decode.decode_skywalking_raw(g["inputs"]))
    _same(anomod.load_trace_file(golden / "jaeger_small.json"),
          decode.decode_jaeger(json.loads((golden / "jaeger_small.json").read_text())))


@pytest.mark.parametrize("seed", range(3))
def test_parallel_decode_equals_one_thread(seed, monkeypatch):
    """Element-parallel decode (structural scan + per-thread parse) gives the
    one-thread columns on large messy dumps and SkyWalking payloads."""
    doc = _messy_jaeger(random.Random(100 + seed), n_traces=900)
    text = json.dumps(doc, indent=2 if seed % 2 else None, ensure_ascii=bool(seed % 3)).encode()
    assert len(text) > 64 << 10
    out = {}
    for th in ("1", "3", "8"):
        monkeypatch.setenv("ANOMOD_DECODE_THREADS", th)
        out[th] = anomod.decode_native(text, "jaeger")
    _same(out["3"], out["1"])
    _same(out["8"], out["1"])
    _same(out["1"], decode.decode_jaeger(json.loads(text)))


def test_parallel_decode_structure_edge_cases(monkeypatch):
    """Shapes the structural scan must get right (or hand to the one-thread
    path): a repeated top-level key (json.load keeps the last), keys and
    strings with escapes / brackets, scalar elements, extra members after the
    array, invalid separators."""
    big = _messy_jaeger(random.Random(7), n_traces=400)["data"]
    first = _messy_jaeger(random.Random(8), n_traces=300)["data"]
    docs = [
        '{"data": %s, "total": 0, "errors": null}' % json.dumps(big),
        '{"x\\"y": "[{", "data": %s, "data": %s}' % (json.dumps(first), json.dumps(big)),
        '{"meta": {"data": [1, 2]}, "data": %s}' % json.dumps(big),
        '{"data": [1, "s", null, %s]}' % json.dumps(big)[1:-1],
        '  {"data": %s}  \n' % json.dumps(big),
    ]
    for k, text in enumerate(docs):
        raw = text.encode()
        monkeypatch.setenv("ANOMOD_DECODE_THREADS", "1")
        one = anomod.decode_native(raw, "jaeger")
        monkeypatch.setenv("ANOMOD_DECODE_THREADS", "8")
        _same(anomod.decode_native(raw, "jaeger"), one)
        if k != 3:  # scalar traces: the reference (and the Python twin) raise on .get
            _same(one, decode.decode_jaeger(json.loads(raw)))
    bad = ['{"data": [%s, ]}' % json.dumps(big)[1:-1], '{"data": [%s}' % json.dumps(big)[1:-1],
           '{"data": %s} x' % json.dumps(big), '{"data": [%s,, 1]}' % json.dumps(big)[1:-1]]
    for text in bad:
        for th in ("1", "8"):
            monkeypatch.setenv("ANOMOD_DECODE_THREADS", th)
            with pytest.raises(anomod.AnomodError):
                anomod.decode_native(text.encode(), "jaeger")


def test_parallel_decode_skywalking(golden, monkeypatch):
    g = json.loads((golden / "skywalking_small.json").read_text())
    payload = dict(g["payload"])
    payload["traces"] = payload["traces"] * 60  # > 64 KiB
    raw = json.dumps(payload, indent=2).encode()
    monkeypatch.setenv("ANOMOD_DECODE_THREADS", "1")
    one = anomod.decode_native(raw, "skywalking")
    monkeypatch.setenv("ANOMOD_DECODE_THREADS", "6")
    _same(anomod.decode_native(raw, "skywalking"), one)
    _same(one, decode.decode_skywalking_payload(payload))
