"""load_experiment -> features -> rank: the engine's call surface.

The reference produces one experiment's telemetry with bash + Python
collectors (SURVEY.md §3 call stacks A-C) and stops at files; this module
reads those files (or a synthetic equivalent) and computes the RCA features
on the GPU:

* edge table: libanomod edge aggregation (HIP), per-edge histogram, counts,
  errors, p50/p99;
* window scores: libanomod EWMA/z kernel over the metric matrix;
* ranking: libanomod personalized PageRank over the caller -> callee graph,
  seeded by per-service anomaly scores.
"""
from __future__ import annotations

import math
import re
import threading
from dataclasses import dataclass, field
from pathlib import Path

import numpy as np

from . import decode
from .device import Context, SynthSpec, synth_generate_host
from .spans import EdgeTable, SpanSet

# --------------------------------------------------------------------------
# Ground-truth labels (experiment name -> faulty service), SURVEY.md §2:
# SN automated_multimodal_collection.sh:904-916 / :323-496;
# TT chaos-experiments/*.yaml target_service and run_experiment.sh:299-345.
# --------------------------------------------------------------------------
_SN_LABELS = {
    "Svc_Kill_Media": "media-service",
    "Svc_Kill_SocialGraph": "social-graph-service",
    "Svc_Kill_UserTimeline": "user-timeline-service",
    "Code_Stop_MediaService": "media-service",
    "Code_Stop_TextService": "text-service",
    "Code_Stop_UserService": "user-service",
    "DB_Redis_CacheLimit_HomeTimeline": "home-timeline-service",
    "DB_Redis_CacheLimit_SocialGraph": "social-graph-service",
    "DB_Redis_CacheLimit_UserTimeline": "user-timeline-service",
}


def fault_target(experiment_name: str) -> str | None:
    """Faulty service named by an experiment directory, if the name encodes one."""
    for key, svc in _SN_LABELS.items():
        if experiment_name.startswith(key):
            return svc
    m = re.search(r"(ts-[a-z0-9-]+-service)", experiment_name)
    if m:
        return m.group(1)
    return None


@dataclass
class Experiment:
    name: str
    spans: SpanSet | None
    metrics: decode.MetricMatrix | None = None
    label: str | None = None
    meta: dict = field(default_factory=dict)

    @property
    def services(self) -> list[str]:
        return self.spans.services if self.spans is not None else []


def _synthetic_metrics(services: list[str], T: int, series_per_service: int, seed: int,
                       fault: str | None) -> decode.MetricMatrix:
    rng = np.random.default_rng(seed)
    keys, cols = [], []
    for s in services:
        for k in range(series_per_service):
            mu, sd = rng.uniform(10, 1000), rng.uniform(0.5, 5)
            x = mu + sd * rng.standard_normal(T)
            if fault is not None and s == fault:
                x[T // 2:] += 8 * sd  # level shift at the fault
            keys.append((f"synthetic_metric_{k}", (("service", s),)))
            cols.append(x.astype(np.float32))
    X = np.stack(cols, axis=1) if cols else np.zeros((T, 0), np.float32)
    return decode.MetricMatrix(X, np.arange(T, dtype=np.float64) * 15.0, keys)


def load_experiment(source, *, metrics=None, name: str | None = None,
                    services: list[str] | None = None, n_traces: int | None = None,
                    metric_steps: int = 480, series_per_service: int = 4) -> Experiment:
    """Load one experiment.

    ``source`` is one of
      * a :class:`SynthSpec` — synthetic SN/TT spans (``n_traces`` traces,
        default 600 = 50 per SN service as collect_trace.sh:18/:49 scrapes)
        over the services they name, plus a synthetic metric matrix;
      * a Jaeger dump (``all_traces.json``) or its directory
        (SN_data/trace_data/<exp>_traces_<ts>/);
      * a SkyWalking payload JSON (TT_data/trace_data/<exp>/*.json) or its
        directory;
    ``metrics`` optionally names an SN metric directory (one CSV per query)
    or a TT long-format metric CSV.
    """
    if isinstance(source, SynthSpec):
        nt = 600 if n_traces is None else n_traces
        spans = synth_generate_host(source, nt)
        fault = source.fault_service
        if isinstance(fault, int):
            fault = spans.services[fault]
        # the services the traces name, as a collector payload lists them
        # (services_discovered, trace_collector.py:572): the same experiment
        # read back from its files has the same service list
        spans = spans.observed_services()
        X = _synthetic_metrics(spans.services, metric_steps, series_per_service,
                               source.seed ^ 0x5EED, fault) if metric_steps else None
        return Experiment(name or f"synthetic_{source.topology}", spans, X, fault,
                          {"synthetic": True})

    path = Path(source)
    exp_name = name or (path.name if path.is_dir() else path.parent.name)
    doc_path = path
    if path.is_dir():
        if (path / "all_traces.json").exists():
            doc_path = path / "all_traces.json"
        else:
            cands = sorted(path.glob("*skywalking_traces_*.json")) or sorted(path.glob("*.json"))
            if not cands:
                raise FileNotFoundError(f"no trace JSON under {path}")
            doc_path = cands[-1]
    # the metric file decodes on a second host thread while the trace file
    # decodes here: both decoders are native and release the GIL, and each
    # has a serial stretch the other's threads fill
    got: dict = {}
    worker = None
    if metrics is not None:
        mp = Path(metrics)

        def _metrics():
            try:
                got["m"] = (decode.decode_prometheus_csv_dir_native(mp) if mp.is_dir()
                            else decode.decode_metric_long_csv_native(mp))
            except BaseException as e:  # noqa: BLE001 (re-raised below)
                got["e"] = e

        worker = threading.Thread(target=_metrics, name="anomod-metrics-decode")
        worker.start()
    try:
        spans = decode.load_trace_file(doc_path, services)
    finally:
        if worker is not None:
            worker.join()
    if "e" in got:
        raise got["e"]
    return Experiment(exp_name, spans, got.get("m"), fault_target(exp_name),
                      {"trace_file": str(doc_path)})


@dataclass
class Features:
    experiment: str
    edges: EdgeTable
    window_scores: np.ndarray | None      # [T/W, S] max |z| per window
    series: list | None
    service_scores: np.ndarray             # [n_services] anomaly score
    params: dict = field(default_factory=dict)


_default_ctx: Context | None = None


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None or _default_ctx.handle is None:
        _default_ctx = Context(0)
    return _default_ctx


def _series_service(key, services: list[str], memo: dict | None = None) -> int | None:
    """Map a metric series to a service by its label values (pod, container,
    service, job ... carry the service name in both datasets): the longest
    service name contained in a label value, the first such in `services`
    order on ties.  Service names hold no spaces, so this is decided value by
    value; `memo` (one per call site) keeps each distinct value's answer."""
    labels = key[1] if len(key) > 1 else ()
    best = None
    for _, v in labels:
        v = str(v)
        hit = memo.get(v, -2) if memo is not None else -2
        if hit == -2:
            hit = -1
            for i, s in enumerate(services):
                if s and s in v and (hit < 0 or len(s) > len(services[hit])):
                    hit = i
            if memo is not None:
                memo[v] = hit
        if hit >= 0 and (best is None or len(services[hit]) > len(services[best])
                         or (len(services[hit]) == len(services[best]) and hit < best)):
            best = hit
    return best


def _latency_shift(cur: EdgeTable, base: EdgeTable, min_count: int = 10) -> np.ndarray:
    """Per service: largest log2 growth of an incoming edge's GPU p99 over
    the same edge — matched by service NAMES (the two runs may have seen
    different service sets: services_discovered lists only the services a
    run's traces name, trace_collector.py:572) — in a baseline run (edges
    with >= min_count spans on both sides)."""
    S, Sb = cur.n_services, base.n_services
    out = np.zeros(S)
    pos = {s: i for i, s in enumerate(base.services)}
    m = np.array([pos.get(s, -1) for s in cur.services] + [Sb, Sb + 1], np.int64)  # + ROOT, ORPHAN
    p_cur = np.repeat(np.arange(S + 2), S)
    c_cur = np.tile(np.arange(S), S + 2)
    pb, cb = m[p_cur], m[c_cur]
    have = (pb >= 0) & (cb >= 0)
    rows = np.where(have, pb * Sb + np.where(cb >= 0, cb, 0), 0)
    bc = np.where(have, base.count[rows], 0)
    bp = np.where(have, base.p99_us[rows], np.nan)
    ok = ((cur.count >= min_count) & (bc >= min_count) & np.isfinite(cur.p99_us)
          & np.isfinite(bp) & (bp > 0))
    ratio = np.zeros(cur.count.shape[0])
    ratio[ok] = np.maximum(0.0, np.log2(cur.p99_us[ok] / bp[ok]))
    return ratio.reshape(S + 2, S).max(axis=0)


def features(exp: Experiment, ctx: Context | None = None, *, W: int = 60,
             alpha: float | None = None, eps: float = 1e-12, with_hist: bool = True,
             baseline: "Features | None" = None) -> Features:
    """GPU features of one experiment (SURVEY.md §3 stack D steps 4-7)."""
    ctx = ctx or default_context()
    edges = ctx.edge_aggregate(exp.spans, with_hist=with_hist)
    S = edges.n_services
    alpha = 2.0 / (W + 1) if alpha is None else alpha
    Z = None
    series = None
    metric_score = np.zeros(S)
    if exp.metrics is not None and exp.metrics.S > 0 and exp.metrics.T > 0:
        mm = exp.metrics.pad_to_multiple(W)
        Z = ctx.ewma_z(mm.X, alpha, W, eps)
        series = mm.series
        # score a series by the mean of its top-5 % window scores (robust to
        # a single spike), then take the max over the series of a service
        k = max(1, Z.shape[0] // 20)
        top = np.sort(Z, axis=0)[-k:].mean(axis=0) if Z.shape[0] else np.zeros(Z.shape[1])
        # series -> service, decided once per distinct label set (a TT matrix
        # holds ~6 k series over ~50 label sets), then one scatter-max
        memo: dict = {}
        labs = [k[1] if len(k) > 1 else () for k in series]
        if not all(isinstance(lb, tuple) for lb in labs):  # a caller's lists of pairs
            labs = [lb if isinstance(lb, tuple) else tuple(tuple(kv) for kv in lb) for lb in labs]
        by_labels = {}
        for lb in dict.fromkeys(labs):
            i = _series_service(("", lb), edges.services, memo)
            by_labels[lb] = -1 if i is None else i
        idx = np.fromiter(map(by_labels.__getitem__, labs), np.int64, len(labs))
        ok = idx >= 0
        np.maximum.at(metric_score, idx[ok], np.asarray(top, np.float64)[ok])
    # error rate of the calls each service serves
    cnt = edges.count.reshape(S + 2, S).sum(axis=0).astype(np.float64)
    err = edges.errors.reshape(S + 2, S).sum(axis=0).astype(np.float64)
    err_rate = np.divide(err, cnt, out=np.zeros(S), where=cnt > 0)
    lat = np.zeros(S)
    if baseline is not None:
        lat = _latency_shift(edges, baseline.edges)
    ms = metric_score / (1.0 + metric_score)  # squash z into [0, 1)
    score = err_rate + lat + 0.25 * ms
    return Features(exp.name, edges, Z, series, score,
                    {"W": W, "alpha": alpha, "eps": eps,
                     "components": {"error_rate": err_rate, "latency": lat, "metric": ms}})


def rank(feats: Features, *, alpha: float = 0.85, iters: int = 100, tol: float = 1e-10,
         ctx: Context | None = None) -> list[tuple[str, float]]:
    """Root-cause ranking: personalized PageRank over the caller -> callee
    graph (weights = call counts), personalization = service anomaly scores."""
    ctx = ctx or default_context()
    services = feats.edges.services
    row_ptr, col, w = feats.edges.call_graph()
    p = np.asarray(feats.service_scores, np.float64).copy()
    if not np.isfinite(p).all() or p.sum() <= 0:
        p = np.ones(len(services))
    p = p + 1e-9 * p.sum()  # every node reachable by the restart
    x, _ = ctx.pagerank(row_ptr, col, w, p, alpha=alpha, iters=iters, tol=tol)
    order = np.argsort(-x, kind="stable")
    return [(services[i], float(x[i])) for i in order]


def hit_at(ranking: list[tuple[str, float]], target: str | None, k: int) -> float | math.nan:
    if target is None:
        return math.nan
    return 1.0 if target in [s for s, _ in ranking[:k]] else 0.0
