"""API-response summaries: monitor_http_responses.py
generate_summary and enhanced_openapi_monitor.py generate_reports.

Goldens: tests/golden/api_summary.json, the reference's own output files for
synthetic responses (tests/golden/gen/make_goldens.py --only api, TZ=UTC).
CPU: the oracle restatement reproduces every file byte for byte.  GPU: the
libanomod path reproduces every field exactly except ``mean`` (device sum
over the sorted values: rtol 1e-12) and the set-ordered ``common_errors``.
"""
import json
import os
import time

import numpy as np
import pytest

from oracle import spec


def _cases(golden):
    cases = json.loads((golden / "api_summary.json").read_text())
    for c in cases:  # JSON turned the int status-code keys into strings
        c["stats"]["status_codes"] = {int(k): v for k, v in c["stats"]["status_codes"].items()}
    return cases


@pytest.fixture(autouse=True)
def _utc():
    old = os.environ.get("TZ")
    os.environ["TZ"] = "UTC"
    time.tzset()
    yield
    if old is None:
        os.environ.pop("TZ")
    else:
        os.environ["TZ"] = old
    time.tzset()


def test_oracle_generate_summary_matches_reference(golden):
    for c in _cases(golden):
        info = c["info"]
        mine = spec.response_summary(c["responses"], info["start_time"], info["duration"],
                                     info["endpoints"])
        assert json.dumps(mine, indent=2) == c["summary_json"]


def test_oracle_generate_reports_matches_reference(golden):
    for c in _cases(golden):
        info = c["info"]
        summ, csv_text, perf = spec.response_reports(
            c["responses"], c["stats"], info["start_time"], info["duration"], info["endpoints"],
            info["sample_interval"])
        ref = c["reports"]
        assert csv_text == ref["status_code_distribution.csv"]
        assert json.dumps(perf, indent=2) == ref["endpoint_performance.json"]
        ref_summ = json.loads(ref["response_summary.json"])
        assert set(summ["error_summary"].pop("common_errors")) == \
            set(ref_summ["error_summary"].pop("common_errors"))
        assert json.loads(json.dumps(summ)) == ref_summ


def _same_stats(mine: dict, ref: dict):
    assert mine.keys() == ref.keys()
    for k, v in ref.items():
        if k.startswith("mean"):
            assert mine[k] == pytest.approx(v, rel=1e-12)
        else:
            assert type(mine[k]) is type(v) and mine[k] == v, k


@pytest.mark.gpu
def test_gpu_generate_summary_matches_reference(ctx, golden, tmp_path):
    import anomod
    for c in _cases(golden):
        info = c["info"]
        f = tmp_path / "s.json"
        assert anomod.api.generate_summary(ctx, c["responses"], f, start_time=info["start_time"],
                                           duration=info["duration"], endpoints=info["endpoints"])
        mine, ref = json.loads(f.read_text()), json.loads(c["summary_json"])
        _same_stats(mine.pop("latency_statistics"), ref.pop("latency_statistics"))
        assert mine == ref
        assert list(mine["content_type_distribution"]) == list(ref["content_type_distribution"])
    assert not anomod.api.generate_summary(ctx, [], tmp_path / "none.json", start_time=0,
                                           duration=1, endpoints=[])
    assert not (tmp_path / "none.json").exists()


@pytest.mark.gpu
def test_gpu_generate_reports_matches_reference(ctx, golden, tmp_path):
    import anomod
    for c in _cases(golden):
        info = c["info"]
        anomod.api.generate_reports(ctx, c["responses"], c["stats"], tmp_path,
                                    start_time=info["start_time"], duration=info["duration"],
                                    endpoints=info["endpoints"],
                                    sample_interval=info["sample_interval"])
        ref = c["reports"]
        for name in ("status_code_distribution.csv", "endpoint_performance.json"):
            assert (tmp_path / name).read_text() == ref[name], name
        mine = json.loads((tmp_path / "response_summary.json").read_text())
        ref_summ = json.loads(ref["response_summary.json"])
        _same_stats(mine.pop("latency_statistics"), ref_summ.pop("latency_statistics"))
        assert set(mine["error_summary"].pop("common_errors")) == \
            set(ref_summ["error_summary"].pop("common_errors"))
        assert mine == ref_summ


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 3, 99, 100, 101, 4097, 300000])
def test_gpu_value_summary_exact_order_statistics(ctx, n):
    """Exact picks vs a host sort at sizes the radix sort tiles differently;
    zeros / negatives / NaN dropped by the positive filter; ties."""
    import anomod
    rng = np.random.default_rng(n)
    v = np.round(rng.lognormal(3, 1.5, n), 2)
    v[rng.random(n) < 0.05] = 0.0
    v[rng.random(n) < 0.01] = -1.0
    v[rng.random(n) < 0.01] = np.nan
    sel = v[v > 0]
    got = anomod.api.value_statistics(ctx, v.tolist())
    if sel.size == 0:
        assert got == {}
        return
    ref = spec.latency_picks(sel.tolist())
    _same_stats(got, ref)
    allv = anomod.api.value_statistics(ctx, np.nan_to_num(v, nan=2.5).tolist(),
                                       positive_only=False, suffix="_ms")
    _same_stats(allv, spec.latency_picks(np.nan_to_num(v, nan=2.5).tolist(), "_ms"))


@pytest.mark.gpu
def test_gpu_value_summary_int_and_mixed_types(ctx):
    import anomod
    ints = [5, 3, 3, 9, 0, 12]
    _same_stats(anomod.api.value_statistics(ctx, ints), spec.latency_picks([5, 3, 3, 9, 12]))
    mixed = [3, 3.0, 2.5, 7, 7.0, 1]  # ties between int and float: stable-sort order
    _same_stats(anomod.api.value_statistics(ctx, mixed), spec.latency_picks(mixed))
    with pytest.raises(ValueError):
        anomod.api.value_statistics(ctx, [1.0, float("nan")], positive_only=False)
