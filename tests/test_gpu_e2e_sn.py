"""End-to-end on files, BASELINE config 1 (SocialNetwork): the reference's call
path writes a Jaeger dump per experiment (collect_trace.sh:54-60 ->
SN_data/trace_data/<exp>_traces_<ts>/all_traces.json, converted at
collect_trace.sh:70) and one CSV per Prometheus query
(fetch_prometheus_metrics.py:99-102 -> SN_data/metric_data/<exp>_metrics_<ts>/).
Here: the golden Jaeger dump (tests/golden/jaeger_small.json) staged as such an
experiment directory and the golden metric directory written by the
reference's own fetch_prometheus_metrics() (tests/golden/prom_dir) ->
load_experiment -> features -> rank on the GPU, each stage checked against the
CPU oracle on the decoded inputs:

* edge table == the C oracle's on the decoded spans (integers bit-exact,
  quantiles identical);
* window scores == the oracle's EWMA/z on the decoded, padded matrix
  (rtol 1e-5: f32 z from f64 state);
* ranking vector within 1e-5 L1 of the oracle's PageRank on the same graph and
  personalization.
"""
import shutil

import numpy as np
import pytest

import anomod
from oracle import native

from test_gpu_edge import assert_table_equal

pytestmark = pytest.mark.gpu

EXP = "Svc_Kill_Media_20251103_230000"


def test_sn_files_to_ranking(ctx, golden, tmp_path):
    d = tmp_path / "trace_data" / f"{EXP}_traces_2025-11-03_23-10-00"
    d.mkdir(parents=True)
    shutil.copy(golden / "jaeger_small.json", d / "all_traces.json")
    mdir = tmp_path / "metric_data" / f"{EXP}_metrics_2025-11-03_23-10-00"
    shutil.copytree(golden / "prom_dir", mdir)

    exp = anomod.load_experiment(d, metrics=mdir, name=EXP)
    assert exp.label == "media-service"
    assert exp.spans.n_spans == 342 and exp.spans.n_traces == 48
    assert (exp.metrics.T, exp.metrics.S) == (36, 9)

    W = 12
    f = anomod.features(exp, ctx, W=W)
    # edge table: GPU == oracle on the decoded spans
    ref = native.finalize(native.edge_aggregate(exp.spans, len(exp.spans.services)))
    assert_table_equal(f.edges, ref)
    assert int(f.edges.count.sum()) == exp.spans.n_spans
    # window scores: GPU EWMA/z == oracle on the same (padded) matrix
    mm = exp.metrics.pad_to_multiple(W)
    Zr = native.ewma_z(mm.X, f.params["alpha"], W, f.params["eps"])
    assert f.window_scores.shape == Zr.shape == (36 // W, 9)
    np.testing.assert_allclose(f.window_scores, Zr, rtol=1e-5, atol=1e-6)
    # ranking: GPU PageRank == oracle on the call graph and personalization
    # rank() builds (same restart smoothing)
    ranking = anomod.rank(f, ctx=ctx)
    row_ptr, col, w = f.edges.call_graph()
    p = np.asarray(f.service_scores, np.float64).copy()
    if not np.isfinite(p).all() or p.sum() <= 0:
        p = np.ones(len(f.edges.services))
    p = p + 1e-9 * p.sum()
    xr, _ = native.pagerank(row_ptr, col, w, p, 0.85, iters=100, tol=1e-10)
    got = dict(ranking)
    x = np.array([got[s] for s in f.edges.services])
    assert np.abs(x - xr).sum() < 1e-5
    assert len(ranking) == len(f.edges.services)
