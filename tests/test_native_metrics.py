"""Native metric-file decoders (csrc/metrics_decode.cpp) against the Python
decoders (anomod/decode.py) — which tests/test_decode.py pins to the files
the reference wrote — on the reference goldens and on fuzzed CSVs.  No GPU."""
import csv
import io
import random
import time

import numpy as np
import pytest

import anomod


def _same(a: anomod.MetricMatrix, b: anomod.MetricMatrix):
    assert a.series == b.series
    np.testing.assert_array_equal(a.timestamps, b.timestamps)
    np.testing.assert_array_equal(a.X, b.X)  # NaN == NaN here


@pytest.fixture
def utc(monkeypatch):
    monkeypatch.setenv("TZ", "UTC")
    time.tzset()
    yield
    monkeypatch.undo()
    time.tzset()


def test_long_csv_golden(golden):
    p = golden / "metric_long.csv"
    _same(anomod.decode_metric_long_csv_native(p), anomod.decode_metric_long_csv(p))


def test_prometheus_dir_golden(golden, utc):
    d = golden / "prom_dir"
    _same(anomod.decode_prometheus_csv_dir_native(d), anomod.decode_prometheus_csv_dir(d))


def _fuzz_long(rng: random.Random, rows: int) -> bytes:
    labels = ["instance", "pod", "namespace", "job", "container", "le", "name"]
    vals = ['ts-order-service-7d9c', 'a,b', 'say "hi"', 'x\ny', '', 'ünï', '10.0.0.1:9100']
    buf = io.StringIO()
    w = csv.writer(buf, lineterminator=rng.choice(["\n", "\r\n"]))
    cols = ["metric_name", "timestamp", "datetime", "value"] + sorted(rng.sample(labels, 5))
    if rng.random() < 0.3:
        cols.append(cols[-1])  # a repeated header name: the last column wins
    w.writerow(cols)
    names = ["up", "process_open_fds", "container_memory_usage_bytes", "node_load1"]
    for _ in range(rows):
        t = 1762178400 + 15 * rng.randrange(40) + rng.choice([0, 0, 0.5, 0.25])
        v = rng.choice(["", "NaN", "inf", "-inf", "1e-7", repr(rng.uniform(-1e9, 1e9)),
                        str(rng.randrange(1000)), " 2.5 "])
        if v == "NaN":
            v = ""
        row = [rng.choice(names), repr(t), "2025-11-03T14:00:00", v]
        row += [rng.choice(vals) for _ in cols[4:]]
        if rng.random() < 0.05:
            row = row[: rng.randrange(2, len(row))]  # short rows
        w.writerow(row)
        if rng.random() < 0.02:
            buf.write("\n")  # blank line
    return buf.getvalue().encode()


@pytest.mark.parametrize("seed", range(12))
def test_long_csv_fuzz(seed, tmp_path):
    data = _fuzz_long(random.Random(seed), 400)
    p = tmp_path / "m.csv"
    p.write_bytes(data)
    _same(anomod.decode_metric_long_csv_native(data), anomod.decode_metric_long_csv(p))


@pytest.mark.parametrize("seed", range(6))
def test_prometheus_dir_fuzz(seed, tmp_path, utc):
    rng = random.Random(seed)
    for f in range(rng.randrange(1, 5)):
        buf = io.StringIO()
        w = csv.writer(buf)
        w.writerow(["timestamp", "value", "metric", "service"])
        for _ in range(rng.randrange(0, 80)):
            sec = rng.randrange(60)
            frac = rng.choice(["", ".500", ".250000", ".123456"])
            ts = f"2025-11-03 22:{rng.randrange(60):02d}:{sec:02d}{frac}"
            v = rng.choice(["", "inf", repr(rng.uniform(0, 1e6)), "3"])
            svc = rng.choice(["media-service", "text-service", ""])
            w.writerow([ts, v, f'service="{svc}"' if svc else "", svc])
        (tmp_path / f"q{f}_{rng.randrange(100)}.csv").write_text(buf.getvalue())
    _same(anomod.decode_prometheus_csv_dir_native(tmp_path),
          anomod.decode_prometheus_csv_dir(tmp_path))


def test_empty_and_header_only(tmp_path):
    for data in (b"", b"metric_name,timestamp,datetime,value\n"):
        m = anomod.decode_metric_long_csv_native(data)
        assert m.T == 0 and m.S == 0


def test_bad_rows_raise():
    with pytest.raises(anomod.AnomodError):
        anomod.decode_metric_long_csv_native(b"metric_name,timestamp,datetime,value\nup,x,y,1\n")
    with pytest.raises(anomod.AnomodError):
        anomod.decode_metric_long_csv_native(b"metric_name,timestamp,datetime,value\nup,1,y,zz\n")


@pytest.mark.parametrize("order", ["series_major", "shuffled"])
def test_long_csv_threaded_pieces_and_fill(order, tmp_path, monkeypatch):
    """A long CSV over the 8-MiB piece threshold (parsed in newline-aligned
    pieces on several threads) with enough samples that the matrix fill runs
    on several threads too (series-rank ranges, every thread walking the
    samples in row order): series with 0, 1 and 2 labels, repeated
    (series, timestamp) rows with other values (the first row must win, also
    when the repeats land in another piece), missing values, rows in series-
    major or shuffled order.  Equal on 1 and 8 threads, and to the Python
    decoder."""
    rng = random.Random(3 if order == "shuffled" else 4)
    cols = ["metric_name", "timestamp", "datetime", "value", "instance", "service"]
    series = [(f"m{k % 37}", f"10.0.0.{k % 7}" if k % 3 else "", f"svc{k % 11}" if k % 5 else "")
              for k in range(1100)]
    rows = []
    for name, inst, svc in series:
        for t in range(0, 15 * 180, 15):
            v = "" if rng.random() < 0.01 else repr(round(rng.uniform(0, 1e4), 6))
            rows.append([name, str(t), "1970-01-01 00:00:00", v, inst, svc])
    dups = [list(r) for r in rng.sample(rows, 8000)]
    for r in dups:
        r[3] = repr(round(rng.uniform(-1e4, 0), 6))  # later rows of a cell: skipped
    rows = rows + dups  # (shuffled: a repeat may come first, and then it is the one kept)
    if order == "shuffled":
        rng.shuffle(rows)
    buf = io.StringIO()
    w = csv.writer(buf, lineterminator="\n")
    w.writerow(cols)
    w.writerows(rows)
    data = buf.getvalue().encode()
    assert len(data) > (8 << 20) + (1 << 20)
    p = tmp_path / "m.csv"
    p.write_bytes(data)
    monkeypatch.setenv("ANOMOD_DECODE_THREADS", "1")
    one = anomod.decode_metric_long_csv_native(p)
    monkeypatch.setenv("ANOMOD_DECODE_THREADS", "8")
    many = anomod.decode_metric_long_csv_native(p)
    _same(many, one)
    _same(one, anomod.decode_metric_long_csv(p))
    assert one.S == len(set(series)) and one.T == 180


@pytest.mark.filterwarnings("ignore:overflow encountered in cast")  # 1.8e308 -> f32 inf
def test_value_and_timestamp_number_forms(tmp_path):
    """The native number parser's fast path (digits[.digits] as one integer
    over a power of ten) and its strtod fallback against Python float() —
    the reference's rule — on the forms a CSV can hold: signs, leading
    zeros, a bare point on either side, exponents, spaces, integers above
    2^53, more than 19 digits, more than 22 fraction digits.  Bit-equal
    (sign of zero included)."""
    vals = ["-0", "0", "0.0", "-0.0", "5.", ".5", "-.5", "00001.5", "1e5", "1E-3", "+3",
            "  7", "7  ", "9007199254740992", "9007199254740993", "18446744073709551617",
            "123456789012345678901", "0.1234567890123456789012", "0.00000000000000000000001",
            "3.14159265358979323846", "-123.456", "1.7976931348623157e308", "inf", "-inf",
            "nan", "2.5e-310", "0.30000000000000004", "1234567890123456.5"]
    rows = ["metric_name,timestamp,datetime,value,service"]
    for k, v in enumerate(vals):
        rows.append(f'up,{k * 15}{".0" if k % 2 else ""},x,"{v}",svc')  # quoted: spaces kept
        rows.append(f"up2,{k}.{k:03d},x,{v.strip()},svc")
    data = ("\n".join(rows) + "\n").encode()
    p = tmp_path / "m.csv"
    p.write_bytes(data)
    nat = anomod.decode_metric_long_csv_native(data)
    ref = anomod.decode_metric_long_csv(p)
    assert nat.series == ref.series
    np.testing.assert_array_equal(nat.timestamps.view(np.uint64), ref.timestamps.view(np.uint64))
    a, b = nat.X.view(np.uint32), ref.X.view(np.uint32)
    nan = np.isnan(nat.X) & np.isnan(ref.X)
    assert np.array_equal(a[~nan], b[~nan])
