"""End-to-end on files, BASELINE config 2 shape (TrainTicket): a SkyWalking
collector payload (trace_collector.py:564-578) and a TT long metric CSV
(metric_collector.py:453-467, written by anomod.write_metric_long_csv) for a
fault experiment and a normal one -> load_experiment -> features (GPU edge
table, EWMA/z) -> rank (GPU PageRank) -> the injected service in the top 3."""
import json

import numpy as np
import pytest

import anomod

pytestmark = pytest.mark.gpu

FAULT = "ts-order-service"


def _payload(sp) -> dict:
    traces = []
    for t in range(sp.n_traces):
        a, b = int(sp.trace_ptr[t]), int(sp.trace_ptr[t + 1])
        node = {int(sp.span_id[i]): f"seg{t}-{i - a}:0" for i in range(a, b)}
        spans = []
        for i in range(a, b):
            pid = int(sp.parent_span_id[i])
            spans.append({
                "trace_id": f"t{t}", "node_id": node[int(sp.span_id[i])],
                "parent_node_id": (node.get(pid, "gone:0") if pid else None),
                "service_code": sp.services[int(sp.svc[i])],
                "start_timestamp_ms": 1762128000000 + t,
                "end_timestamp_ms": 1762128000000 + t + int(sp.dur_us[i]) // 1000,
                "is_error": bool(sp.flags[i] & anomod.FLAG_ERROR)})
        traces.append({"summary": {"trace_id": f"t{t}"}, "span_count": b - a, "spans": spans})
    return {"metadata": {"services_discovered": sorted(sp.services)}, "traces": traces}


def _metric_results(services, fault, seed, T=480):
    rng = np.random.default_rng(seed)
    ts = 1762128000 + 15 * np.arange(T)
    out = {}
    for q in ("container_cpu_usage_seconds_total", "container_memory_working_set_bytes"):
        res = []
        for s in services:
            mu, sd = rng.uniform(10, 1000), rng.uniform(0.5, 5)
            x = mu + sd * rng.standard_normal(T)
            if s == fault and q.startswith("container_cpu"):
                x[T // 2:] += 8 * sd
            res.append({"metric": {"__name__": q, "container": s, "pod": f"{s}-7d9f-x"},
                        "values": [[float(t), repr(float(v))] for t, v in zip(ts, x)]})
        out[q] = res
    return out


def _write_experiment(tmp, name, fault, seed):
    sp = anomod.synth_generate_host(anomod.SynthSpec("TT", seed=seed, fault_service=fault), 4000)
    d = tmp / name
    d.mkdir()
    (d / f"{name}_skywalking_traces_1.json").write_text(json.dumps(_payload(sp), indent=2))
    csv_path = tmp / f"{name}_metrics.csv"
    anomod.write_metric_long_csv(_metric_results(sp.services, fault, seed), csv_path)
    return d, csv_path


def test_tt_files_to_ranking(ctx, tmp_path):
    nd, nm = _write_experiment(tmp_path, "normal_1", None, 41)
    fd, fm = _write_experiment(tmp_path, f"{FAULT}_cpu_1", FAULT, 42)
    base = anomod.load_experiment(nd, metrics=nm)
    exp = anomod.load_experiment(fd, metrics=fm)
    assert exp.label == FAULT and exp.spans.n_traces == 4000
    assert exp.metrics.S == 2 * len(anomod.synth_services("TT")) and exp.metrics.T == 480
    fb = anomod.features(base, ctx)
    fe = anomod.features(exp, ctx, baseline=fb)
    assert int(fe.edges.count.sum()) == exp.spans.n_spans
    assert fe.window_scores.shape == (480 // 60, exp.metrics.S)
    ranking = anomod.rank(fe, ctx=ctx)
    assert anomod.hit_at(ranking, FAULT, 3) == 1.0


def test_tt_files_rank_as_memory(ctx, tmp_path):
    """Config 2 from files == config 2 from memory on the GPU: the staged
    experiment (whole-ms durations, services_discovered) gives the in-memory
    edge table bit for bit and the same ranking vector, with the same
    baseline on both sides."""
    from test_tt_file_roundtrip import stage

    from test_gpu_edge import assert_table_equal

    base_m, bd, bm = stage(tmp_path, i=0, fault=None)
    exp_m, fd, fm = stage(tmp_path, i=3, fault="ts-order-service")
    base_f = anomod.load_experiment(bd, metrics=bm)
    exp_f = anomod.load_experiment(fd, metrics=fm)
    fb_m, fb_f = anomod.features(base_m, ctx), anomod.features(base_f, ctx)
    fe_m = anomod.features(exp_m, ctx, baseline=fb_m)
    fe_f = anomod.features(exp_f, ctx, baseline=fb_f)
    assert fe_f.edges.services == fe_m.edges.services
    ref = {k: getattr(fe_m.edges, k) for k in ("count", "errors", "sum_us", "min_us", "max_us",
                                               "hist")}
    assert_table_equal(fe_f.edges, ref)
    np.testing.assert_array_equal(fe_f.service_scores, fe_m.service_scores)
    assert anomod.rank(fe_f, ctx=ctx) == anomod.rank(fe_m, ctx=ctx)
