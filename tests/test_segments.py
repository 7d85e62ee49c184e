"""Segment summary: host decoding against the
reference's extract_trace_info outputs, and the GPU reductions against the
reference's analyze_trace_patterns result (tests/golden/analyze_patterns.json,
written by tests/golden/gen/make_goldens.py running the reference)."""
import json

import numpy as np
import pytest

import anomod
from oracle import spec


def _golden(golden):
    return json.loads((golden / "analyze_patterns.json").read_text())


def test_decode_matches_extract_trace_info(golden):
    g = _golden(golden)
    infos = anomod.trace_infos(g["segments"])
    assert len(infos) == len(g["traces"])
    for mine, ref in zip(infos, g["traces"]):
        for k in ("service_name", "endpoint_name", "latency", "is_error", "start_time"):
            assert mine[k] == ref[k], k


def test_segment_set_columns(golden):
    g = _golden(golden)
    seg = anomod.SegmentSet.from_es(g["segments"])
    assert seg.n == len(g["traces"])
    assert sorted(seg.services) == g["analysis"]["unique_services"]
    assert [seg.services[i] for i in seg.svc] == [t["service_name"] for t in g["traces"]]
    assert int(seg.is_error.sum()) == g["analysis"]["error_traces"]


def _compare(mine, ref):
    for k in ("total_traces", "error_traces", "service_call_counts", "endpoint_call_counts"):
        assert mine[k] == ref[k], k
    assert sorted(mine["unique_services"]) == sorted(ref["unique_services"])
    assert sorted(mine["unique_endpoints"]) == sorted(ref["unique_endpoints"])
    if isinstance(ref["latency_stats"], dict):
        for k in ("min", "max", "count"):
            assert mine["latency_stats"][k] == ref["latency_stats"][k], k
        assert mine["latency_stats"]["avg"] == ref["latency_stats"]["avg"]
    else:
        assert mine["latency_stats"] == ref["latency_stats"]
    assert mine["time_range"]["earliest"] == ref["time_range"]["earliest"]
    assert mine["time_range"]["latest"] == ref["time_range"]["latest"]


@pytest.mark.gpu
def test_gpu_summary_matches_reference(ctx, golden):
    g = _golden(golden)
    _compare(anomod.analyze_trace_patterns(g["segments"], ctx), g["analysis"])
    _compare(anomod.analyze_trace_patterns(g["traces"], ctx), g["analysis"])


@pytest.mark.gpu
def test_gpu_summary_edge_cases(ctx):
    assert anomod.analyze_trace_patterns([], ctx)["latency_stats"] is None
    t = [{"service_name": "a", "endpoint_name": "x", "latency": 0, "is_error": True,
          "start_time": 0}, {"service_name": "b", "latency": -5, "is_error": 2}]
    mine = anomod.analyze_trace_patterns(t, ctx)
    _compare(mine, spec.analyze_trace_patterns(t))
    assert mine["latency_stats"] == [] and mine["error_traces"] == 1


@pytest.mark.gpu
def test_gpu_summary_large_random(ctx):
    rng = np.random.default_rng(2)
    n = 3_000_000
    svcs = [f"ts-svc-{i}" for i in range(46)]
    eps = [f"GET:/api/{i}" for i in range(5000)]  # more endpoints than LDS ids
    seg = anomod.SegmentSet(svcs, eps, rng.integers(0, 46, n).astype(np.uint32),
                            rng.integers(0, 5000, n).astype(np.uint32),
                            rng.integers(0, 3, n).astype(np.int32),
                            rng.integers(-10, 10**6, n).astype(np.int64),
                            np.where(rng.random(n) < 0.05, 0,
                                     rng.integers(1, 2**41, n)).astype(np.int64))
    got = ctx.segment_summary(seg)
    assert got["service_call_counts"] == {s: int(c) for s, c in
                                          zip(svcs, np.bincount(seg.svc, minlength=46))}
    assert got["endpoint_call_counts"] == {e: int(c) for e, c in
                                           zip(eps, np.bincount(seg.endpoint, minlength=5000))}
    assert got["error_traces"] == int((seg.is_error == 1).sum())
    pos = seg.latency[seg.latency > 0]
    assert got["latency_stats"]["count"] == pos.size
    assert got["latency_stats"]["min"] == int(pos.min())
    assert got["latency_stats"]["max"] == int(pos.max())
    assert got["latency_stats"]["avg"] == int(pos.sum()) / pos.size
    st = seg.start_time[seg.start_time != 0]
    assert got["time_range"]["earliest"] == int(st.min())
    assert got["time_range"]["latest"] == int(st.max())
