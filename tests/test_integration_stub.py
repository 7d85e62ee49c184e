"""INTEGRATION.md §2's reference-side ctypes stub, extracted and run as a
maintainer would drop it next to collect_trace.sh:70: its columns (libanomod's
native Jaeger decoder, CPU) equal anomod.decode's Python restatement of
jaeger_to_csv.py:34-46,55-67,83 — error flags included, on tags chosen to
separate an integer status compare from a string one — and its edge table
(GPU) equals the C oracle's."""
import json
import re
import types

import numpy as np
import pytest

import anomod
from anomod import _lib as L
from anomod.decode import decode_jaeger

from conftest import GOLDEN, ROOT


def _stub() -> types.ModuleType:
    text = (ROOT / "INTEGRATION.md").read_text()
    sec = text[text.index("## 2. ctypes stub"):]
    code = re.search(r"```python\n(.*?)```", sec, re.S).group(1)
    assert "anomod_decode_jaeger" in code and "anomod_edge_aggregate" in code
    mod = types.ModuleType("anomod_features")
    mod.__dict__["__name__"] = "anomod_features"  # not __main__: the CLI block stays off
    import os

    saved = os.environ.get("ANOMOD_LIB")
    os.environ["ANOMOD_LIB"] = str(L.LIB_PATH)  # the stub's one configurable
    try:
        exec(compile(code, "INTEGRATION.md#anomod_features", "exec"), mod.__dict__)
    finally:
        if saved is None:
            del os.environ["ANOMOD_LIB"]
        else:
            os.environ["ANOMOD_LIB"] = saved
    return mod


def _tricky_doc() -> dict:
    """Spans whose tags separate the integer rule from a string compare:
    "60" >= "500" as strings, 1000 < "500" as a string, "503.0" is no int,
    "true" strings and TRUE count, False / "false" do not."""
    cases = [("http.status_code", "60"), ("http.status_code", 1000), ("http.status_code", "503.0"),
             ("http.status_code", "abc"), ("http.status_code", 499), ("http.status_code", "500"),
             ("error", "true"), ("error", "TRUE"), ("error", False), ("error", "false"),
             ("error", True), ("http.status_code", 200)]
    spans = []
    for i, (k, v) in enumerate(cases):
        refs = [] if i == 0 else [{"refType": "CHILD_OF", "traceID": "t1",
                                   "spanID": f"{i:x}"}]
        spans.append({"traceID": "t1", "spanID": f"{i + 1:x}", "operationName": "op",
                      "references": refs, "startTime": 1700000000000000 + i, "duration": 100 + i,
                      "tags": [{"key": k, "type": "string", "value": v}], "logs": [],
                      "processID": f"p{i % 3}"})
    return {"data": [{"traceID": "t1", "spans": spans,
                      "processes": {f"p{j}": {"serviceName": f"svc-{j}"} for j in range(3)}}]}


@pytest.fixture(scope="module")
def stub():
    return _stub()


@pytest.mark.parametrize("which", ["golden", "tricky"])
def test_stub_columns_equal_product_decoder(stub, tmp_path, which):
    if which == "golden":
        path = GOLDEN / "jaeger_small.json"
    else:
        path = tmp_path / "tricky.json"
        path.write_text(json.dumps(_tricky_doc()))
    services, cols, trace_ptr = stub.jaeger_columns(str(path))
    want = decode_jaeger(json.loads(path.read_text()))
    assert services == list(want.services)
    np.testing.assert_array_equal(trace_ptr, want.trace_ptr)
    for k in ("span_id", "parent_span_id", "svc", "flags", "dur_us"):
        np.testing.assert_array_equal(cols[k], getattr(want, k), err_msg=k)
    if which == "tricky":  # 1000, "500", "true", "TRUE", True err; "60" (a string compare
        # would say >= "500"), 499, "503.0" / "abc" (no int), False, "false", 200 do not
        assert cols["flags"].tolist() == [0, 1, 0, 0, 0, 1, 1, 1, 0, 0, 1, 0]


@pytest.mark.gpu
def test_stub_edge_table_equals_oracle(stub):
    from oracle import native

    services, cols, trace_ptr = stub.jaeger_columns(str(GOLDEN / "jaeger_small.json"))
    got = stub.edge_table(services, cols, trace_ptr)
    spans = anomod.SpanSet(services, trace_ptr, cols["trace_hash"], cols["span_id"],
                           cols["parent_span_id"], cols["svc"], cols["flags"], cols["dur_us"])
    ref = native.finalize(native.edge_aggregate(spans))
    for k in ("count", "errors", "sum_us", "min_us", "max_us", "hist"):
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    np.testing.assert_array_equal(got["p50_us"], ref["p50_us"])
    np.testing.assert_array_equal(got["p99_us"], ref["p99_us"])
    assert int(got["count"].sum()) == len(cols["span_id"])
