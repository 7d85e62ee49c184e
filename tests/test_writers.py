"""File-boundary writers byte-equal to the files the
reference's own code wrote (tests/golden: jaeger_small.csv / jaeger_empty.csv
from jaeger_to_csv.py, metric_long.csv from metric_collector.py), and the
metric decoder read back against the Prometheus results those files came
from.  All under TZ=UTC (the goldens were written with TZ=UTC)."""
import json
import math
import time

import numpy as np
import pytest

import anomod
from anomod import writers


@pytest.fixture(autouse=True)
def utc(monkeypatch):
    monkeypatch.setenv("TZ", "UTC")
    time.tzset()
    yield
    time.tzset()


def test_jaeger_csv_byte_equal_to_reference(golden, tmp_path):
    doc = json.loads((golden / "jaeger_small.json").read_text())
    out = tmp_path / "all_traces.csv"
    n = writers.write_jaeger_csv(doc, out)
    assert n > 100
    assert out.read_bytes() == (golden / "jaeger_small.csv").read_bytes()


def test_jaeger_csv_empty_and_cli(golden, tmp_path, capsys):
    (tmp_path / "e.json").write_text('{"data": []}')
    assert writers.jaeger_to_csv(tmp_path / "e.json", tmp_path / "e.csv") == 0
    assert (tmp_path / "e.csv").read_bytes() == (golden / "jaeger_empty.csv").read_bytes()
    (tmp_path / "bad.json").write_text("{not json")
    assert writers.jaeger_to_csv(tmp_path / "bad.json", tmp_path / "b.csv") == 1
    assert "invalid JSON" in capsys.readouterr().out


def test_jaeger_csv_column_typing():
    doc = {"data": [{"traceID": "t", "processes": {"p": {"serviceName": "s"}}, "spans": [
        {"spanID": "a", "duration": 5, "startTime": 1762207158839501,
         "tags": [{"key": "http.status_code", "value": 200}]},
        {"spanID": "b", "duration": 7.5, "startTime": 1762207158839502,
         "tags": [{"key": "http.status_code", "value": 503.0}]}]}]}
    text = writers.to_text(writers.write_jaeger_csv, doc).splitlines()
    # duration and status columns hold a float -> pandas prints them as floats
    assert text[1].split(",")[6:8] == ["5.0", "200.0"]
    assert text[2].split(",")[6:8] == ["7.5", "503.0"]


def test_metric_long_csv_byte_equal_to_reference(golden, tmp_path):
    res = json.loads((golden / "metric_results.json").read_text())
    out = tmp_path / "m.csv"
    writers.write_metric_long_csv(res, out)
    assert out.read_bytes() == (golden / "metric_long.csv").read_bytes()


def test_metric_decoder_reads_reference_csv(golden):
    res = json.loads((golden / "metric_results.json").read_text())
    mm = anomod.decode_metric_long_csv(golden / "metric_long.csv")
    # every (query, labels, timestamp) sample of the source results lands in X
    col = {k: j for j, k in enumerate(mm.series)}
    row = {t: i for i, t in enumerate(mm.timestamps.tolist())}
    seen = 0
    for query, result in res.items():
        for s in result:
            labels = tuple(sorted((k, v) for k, v in s.get("metric", {}).items()
                                  if k != "__name__" and v))
            j = col[(query, labels)]
            for ts, v in s["values"]:
                x = mm.X[row[float(ts)], j]
                if v == "NaN":
                    assert math.isnan(x)
                else:
                    assert x == np.float32(float(v))
                seen += 1
    assert seen == 97 and mm.S == 9
