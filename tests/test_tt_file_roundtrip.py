"""BASELINE config 2 from files reproduces config 2 from memory.

The synthetic TrainTicket topology records whole milliseconds, as SkyWalking
does (duration = end_ms - start_ms, trace_collector.py:87; the decoder reads
ms x 1000).  An experiment staged in the dataset's layout — the collector
payload (trace_collector.py:564-581, json indent=2) and the long metric CSV
(metric_collector.py:453-467) — and read back by load_experiment (native
decoders) must give the in-memory experiment's span columns (services,
flags, durations, trace bounds, parent structure) and metric matrix exactly.
CPU only; the GPU half (identical edge tables and rankings) is in
tests/test_gpu_e2e_tt.py.
"""
import json

import numpy as np
import pytest

import anomod
from anomod import writers


def stage(tmp_path, i=3, fault="ts-order-service", n_traces=300):
    name = f"tt_{i:02d}_{fault}"
    exp = anomod.load_experiment(anomod.SynthSpec("TT", seed=20251103 + i, fault_service=fault),
                                 n_traces=n_traces, series_per_service=3, name=name)
    d = tmp_path / name
    d.mkdir()
    (d / f"{name}_skywalking_traces_20251103_140200.json").write_text(
        json.dumps(writers.skywalking_payload(exp.spans, name), indent=2), encoding="utf-8")
    mc = d / f"{name}_metrics_20251103_140200.csv"
    writers.write_metric_long_csv_matrix(exp.metrics.X, exp.metrics.timestamps,
                                         exp.metrics.series, mc)
    return exp, d, mc


def parent_pos(sp):
    """Per span: position in its trace of the first span whose id equals its
    parent reference (-1: none / not in the trace) — the parent structure,
    independent of how ids are spelled."""
    out = np.full(sp.n_spans, -1, np.int64)
    for t in range(sp.n_traces):
        a, b = int(sp.trace_ptr[t]), int(sp.trace_ptr[t + 1])
        first = {}
        for i in range(a, b):
            first.setdefault(int(sp.span_id[i]), i - a)
        for i in range(a, b):
            p = int(sp.parent_span_id[i])
            out[i] = first.get(p, -1) if p else -1
    return out


def test_tt_durations_are_whole_ms():
    sp = anomod.synth_generate_host(anomod.SynthSpec("TT", seed=5, fault_service=3,
                                                     fault_latency_mult=7), 2000)
    assert (sp.dur_us % 1000 == 0).all()
    assert 0.0 < (sp.dur_us == 0).mean() < 0.15  # some sub-ms spans record 0 ms, as in SkyWalking


def test_tt_files_reproduce_memory(tmp_path):
    exp, d, mc = stage(tmp_path)
    got = anomod.load_experiment(d, metrics=mc)
    a, b = exp.spans, got.spans
    assert got.label == "ts-order-service"
    assert b.services == a.services
    assert b.n_traces == a.n_traces and b.n_spans == a.n_spans
    np.testing.assert_array_equal(b.trace_ptr, a.trace_ptr)
    for k in ("svc", "flags", "dur_us"):
        np.testing.assert_array_equal(getattr(b, k), getattr(a, k), err_msg=k)
    np.testing.assert_array_equal(parent_pos(b), parent_pos(a))
    ma, mb = exp.metrics, got.metrics
    np.testing.assert_array_equal(mb.timestamps, ma.timestamps)
    assert sorted(mb.series) == sorted(ma.series)
    col = {k: j for j, k in enumerate(ma.series)}
    order = [col[k] for k in mb.series]
    np.testing.assert_array_equal(mb.X, ma.X[:, order])
