#!/usr/bin/env python3
"""Headline benchmark: spans/s aggregated into bit-exact call-graph edge
histograms (+ % of HBM peak), with RCA PageRank iters/s and EWMA/z
samples/s alongside (BASELINE.json metric).

One process per GPU.  N=1:  python bench.py
N>1 (driver):  python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
               --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

Each rank generates its own shard of synthetic DeathStarBench-SocialNetwork
spans directly in HBM (generation is outside the
timed region), runs K aggregation steps and — for N > 1 — the RCCL
all-reduce of the integer edge table inside every step.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
PKG_DIR = ROOT / "anomod-a-dataset-for-anomaly-detection-and-root-cause-analysis-in-microservice-systems_amd"
for _p in (str(PKG_DIR), str(ROOT)):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

import anomod  # noqa: E402
from anomod import _lib as L  # noqa: E402

LEGS = ("general_scan", "trace_structure", "exact_quantiles", "in_trace_shuffled", "ungrouped",
        "tt_width", "long_traces", "pagerank", "ewma", "tt_config2", "tt_config2_files")
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip parameters)
METRIC = "spans/sec aggregated (node) + % HBM peak; RCA PageRank iters/sec at 1/2/4/8 GPUs"


def algorithmic_bytes(n_spans: int, n_traces: int) -> int:
    """Bytes the edge-aggregation kernel must read once: span_id 8 +
    parent_span_id 8 + svc 2 + flags 2 + dur_us 4 = 24 B/span, plus the
    8-B trace_ptr entries (trace_hash only picks the shard: not read)."""
    return 24 * n_spans + 8 * (n_traces + 1)


def host_cores() -> dict:
    """CPUs this process may use: the affinity mask, capped by a cgroup v2
    CPU quota and by the box's declared CPU share (OMP_NUM_THREADS, which
    the GPU pool sets to the per-GPU share of a larger machine)."""
    affinity = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    share = os.environ.get("OMP_NUM_THREADS")
    share = int(share) if share and share.isdigit() and int(share) > 0 else None
    usable = affinity
    for cap in (quota, share):
        if cap is not None:
            usable = min(usable, max(1, int(cap)))
    return {"nproc": os.cpu_count(), "affinity": affinity, "cgroup_quota_cores": quota,
            "declared_share": share, "usable": usable}


def _time_oracle(sample, S: int, threads: int, min_seconds: float) -> tuple[int, float]:
    """Passes of the C oracle over the sample on `threads` threads (one trace
    range each; ctypes drops the GIL) until min_seconds have elapsed."""
    from oracle import native

    bounds = np.linspace(0, sample.n_traces, threads + 1).astype(np.int64)
    return _threads_run(
        lambda i: native.edge_aggregate(sample, S, int(bounds[i]), int(bounds[i + 1])), threads,
        min_seconds)


def cpu_baseline(spec, n_traces: int, min_seconds: float) -> dict:
    """The C oracle (oracle/liboracle.so) on every usable host core over a
    bounded sample of the same synthetic workload, plus a one-core figure
    (all-cores and single-core, core count stated)."""
    from oracle import native

    sample = anomod.synth_generate_host(spec, n_traces)
    S = len(sample.services)
    native.lib()
    cores = host_cores()
    threads = cores["usable"]
    passes, el = _time_oracle(sample, S, threads, min_seconds)
    p1, el1 = _time_oracle(sample, S, 1, max(2.0, min_seconds / 3))
    return {"value": sample.n_spans * passes / el, "unit": "spans/s", "cores": threads,
            "kind": "port", "single_core": sample.n_spans * p1 / el1, "host": cores,
            "sample": f"{sample.n_spans} synthetic SN spans ({n_traces} traces) x {passes} "
                      f"passes in {el:.1f} s, C oracle, {threads} threads (every usable core); "
                      f"single core: {p1} passes in {el1:.1f} s"}


def _threads_run(fn, threads: int, min_seconds: float) -> tuple[int, float]:
    """Rounds of fn(i) on `threads` threads (ctypes calls drop the GIL) until
    min_seconds have elapsed -> (rounds, seconds)."""
    rounds, t0 = 0, time.perf_counter()
    while True:
        ts = [threading.Thread(target=fn, args=(i,)) for i in range(threads)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        rounds += 1
        el = time.perf_counter() - t0
        if el >= min_seconds:
            return rounds, el


def cpu_trace_structure(spec, n_traces: int, min_seconds: float) -> dict:
    """C oracle trace structure (oracle_trace_structure) over a host sample of
    the headline workload, one trace range per thread, every usable core."""
    from oracle import native

    sample = anomod.synth_generate_host(spec, n_traces)
    threads = host_cores()["usable"]
    bounds = np.linspace(0, sample.n_traces, threads + 1).astype(np.int64)
    parts = [sample.select_traces((np.arange(sample.n_traces) >= bounds[i])
                                  & (np.arange(sample.n_traces) < bounds[i + 1]))
             for i in range(threads)]
    native.trace_structure(parts[0])  # load
    r, el = _threads_run(lambda i: native.trace_structure(parts[i]), threads, min_seconds)
    return {"value": sample.n_spans * r / el, "unit": "spans/s", "cores": threads, "kind": "port",
            "sample": f"{sample.n_spans} synthetic SN spans ({n_traces} traces) x {r} passes in "
                      f"{el:.1f} s, C oracle_trace_structure, {threads} threads"}


def cpu_group(spec, n_traces: int, min_seconds: float) -> dict:
    """The ungrouped step on the CPU, every usable core: the C oracle's
    grouping (oracle_group_by_trace: a parallel two-level radix partition of
    mix64(trace_hash), spans of a trace in arrival order — spec.group_by_trace
    restated), the gather of the span columns (oracle_take_spans, one row range
    per thread) and the edge table over the grouped spans (oracle_edge_aggregate,
    one trace range per thread, tables summed) — the CPU side of the GPU leg's
    group + join + table step, on an interleaved host sample of the same
    workload."""
    from types import SimpleNamespace

    from oracle import native

    sample = anomod.synth_generate_host(spec, n_traces)
    S = len(sample.services)
    perm = np.random.default_rng(1).permutation(sample.n_spans)
    src = [np.ascontiguousarray(getattr(sample, k)[perm]) for k in
           ("trace_hash", "span_id", "parent_span_id", "svc", "flags", "dur_us")]
    dst = [np.empty_like(a) for a in src]
    threads = host_cores()["usable"]
    n = sample.n_spans
    rows = [(n * i // threads, n * (i + 1) // threads) for i in range(threads)]
    lib = native.lib()

    def step():
        order, tptr = native.group_by_trace(src[0], threads)
        o = np.ascontiguousarray(order, np.uint64)
        _threads_run(lambda i: lib.oracle_take_spans(
            native._p(o), rows[i][0], rows[i][1], *[native._p(a) for a in src],
            *[native._p(a) for a in dst]), threads, 0.0)
        g = SimpleNamespace(services=sample.services, span_id=dst[1], parent_span_id=dst[2],
                            svc=dst[3], flags=dst[4], dur_us=dst[5], trace_ptr=tptr,
                            n_traces=tptr.shape[0] - 1)
        tb = np.linspace(0, g.n_traces, threads + 1).astype(np.int64)
        tabs = [None] * threads

        def agg(i):
            tabs[i] = native.edge_aggregate(g, S, int(tb[i]), int(tb[i + 1]))

        _threads_run(agg, threads, 0.0)
        return sum(t["count"] for t in tabs)

    cnt = step()  # load + warm; every span lands in the table once
    if int(cnt.sum()) != n:
        raise RuntimeError("cpu ungrouped step lost spans")
    r, t0 = 0, time.perf_counter()
    while True:
        step()
        r += 1
        el = time.perf_counter() - t0
        if el >= min_seconds:
            break
    return {"value": n * r / el, "unit": "spans/s", "cores": threads, "kind": "port",
            "sample": f"{n} interleaved synthetic SN spans x {r} ungrouped steps in {el:.1f} s "
                      f"(C oracle: oracle_group_by_trace radix partition + oracle_take_spans + "
                      f"oracle_edge_aggregate, {threads} threads each)"}


def cpu_ewma(T: int, S_slice: int, W: int, min_seconds: float) -> dict:
    """C oracle EWMA/z (oracle_ewma_z) on a [T][S_slice] slice of config 4's
    series, one slice per thread: samples/s, scaled from the slice."""
    from oracle import native

    rng = np.random.default_rng(7)
    X = (100.0 + 5.0 * rng.standard_normal((T, S_slice))).astype(np.float32)
    threads = host_cores()["usable"]
    native.ewma_z(X[:W], 2 / (W + 1), W)
    r, el = _threads_run(lambda i: native.ewma_z(X, 2 / (W + 1), W), threads, min_seconds)
    return {"value": T * S_slice * threads * r / el, "unit": "samples/s", "cores": threads,
            "kind": "port",
            "sample": f"[{T}][{S_slice}] f32 slice of config 4 per thread x {r} rounds in {el:.1f} s, "
                      f"C oracle_ewma_z (f64 state), {threads} threads; the GPU leg is S = 10^5 x "
                      f"T ~ 10^6"}


def cpu_pagerank(N: int, iters: int, seed: int, min_seconds: float) -> dict:
    """C oracle PageRank (oracle_pagerank) on the very synthetic graph the GPU
    leg solves (anomod.synth_graph_csr), one independent solve per thread
    (the replica mode of the GPU leg): solved iterations/s."""
    from oracle import native

    rp, col, w = anomod.synth_graph_csr(N, 10, seed)
    p = np.random.default_rng(0).random(N)
    threads = host_cores()["usable"]
    r, el = _threads_run(lambda i: native.pagerank(rp, col, w, p, iters=iters, tol=0.0), threads,
                         min_seconds)
    return {"value": iters * threads * r / el, "unit": "iters/s", "cores": threads, "kind": "port",
            "sample": f"N = {N}, {col.shape[0]} edges, {iters}-iteration solves x {threads} "
                      f"threads x {r} rounds in {el:.1f} s, C oracle_pagerank"}


# Chaos targets of the TrainTicket runs (chaos-experiments/*.yaml target_service
# labels, run_experiment.sh:299-345); None = the normal run (baseline).
TT_FAULTS = [None, "ts-preserve-service", "ts-order-service", "ts-security-service",
             "ts-travel-service", "ts-auth-service", "ts-basic-service", "ts-route-service",
             "ts-seat-service", "ts-station-service", "ts-price-service",
             "ts-train-service", "ts-user-service"]


def tt_config2(ctx) -> dict:
    """BASELINE config 2 on one GPU: the TrainTicket trace set of 13
    experiments (~15k spans each, 46 services) + their metric matrices
    (S = 5980 series x T = 480 steps @15 s), each taken through the product
    call surface features() -> rank() (H2D of spans and series, edge table,
    EWMA/z, PageRank, D2H and the host glue all inside the timed loop).
    Inputs are synthetic and built in host memory before the clock starts."""
    exps = [anomod.load_experiment(anomod.SynthSpec("TT", seed=20251103 + i, fault_service=f),
                                   n_traces=650, series_per_service=130,
                                   name=f"tt_{f or 'normal'}")
            for i, f in enumerate(TT_FAULTS)]
    base = anomod.features(exps[0], ctx)  # normal run: latency baseline (and warm-up)
    for e in exps[1:3]:
        anomod.rank(anomod.features(e, ctx, baseline=base), ctx=ctx)
    t0 = time.perf_counter()
    base = anomod.features(exps[0], ctx)
    hits = []
    for e in exps[1:]:
        ranking = anomod.rank(anomod.features(e, ctx, baseline=base), ctx=ctx)
        hits.append(anomod.hit_at(ranking, e.label, 3))
    el = time.perf_counter() - t0
    spans = sum(e.spans.n_spans for e in exps)
    samples = sum(e.metrics.S * e.metrics.T for e in exps)
    return {"experiments": len(exps), "spans": spans, "series": exps[0].metrics.S,
            "steps": exps[0].metrics.T, "seconds": el, "ms_per_experiment": el / len(exps) * 1e3,
            "spans_per_s": spans / el, "samples_per_s": samples / el,
            "top3_hit_rate": float(np.mean(hits)),
            "note": "end to end through features()/rank(): host-latency-bound at this size"}


def _stage_tt_experiment(args) -> tuple[str, str, str | None]:
    """Write one synthetic TrainTicket experiment in the dataset's layout:
    <dir>/<exp>/<exp>_skywalking_traces_<ts>.json (the collector payload,
    json.dump indent=2: trace_collector.py:564-581) and <exp>_metrics_<ts>.csv
    (the long CSV of metric_collector.py:453-467)."""
    root, i, fault = args
    from anomod import writers

    name = f"tt_{i:02d}_{fault or 'normal'}"
    exp = anomod.load_experiment(anomod.SynthSpec("TT", seed=20251103 + i, fault_service=fault),
                                 n_traces=650, series_per_service=130, name=name)
    d = Path(root) / name
    d.mkdir(parents=True, exist_ok=True)
    tj = d / f"{name}_skywalking_traces_20251103_140200.json"
    tj.write_text(json.dumps(writers.skywalking_payload(exp.spans, name), indent=2,
                             ensure_ascii=False), encoding="utf-8")
    mc = d / f"{name}_metrics_20251103_140200.csv"
    writers.write_metric_long_csv_matrix(exp.metrics.X, exp.metrics.timestamps,
                                         exp.metrics.series, mc)
    return str(d), str(mc), fault


def stage_tt_files(root: str) -> list:
    """The 13 TT experiments of tt_config2 as files, written by a process
    pool (forked before this process touches the GPU)."""
    import multiprocessing as mp

    work = [(root, i, f) for i, f in enumerate(TT_FAULTS)]
    with mp.get_context("fork").Pool(min(len(work), max(1, host_cores()["usable"]))) as pool:
        return pool.map(_stage_tt_experiment, work)


def _evict_page_cache(paths) -> int:
    """Drop the page-cache pages of these files (fsync, then
    posix_fadvise(DONTNEED); best effort: a tmpfs keeps them).  Returns the
    files handled."""
    done = 0
    for p in paths:
        try:
            fd = os.open(p, os.O_RDONLY)
        except OSError:
            continue
        try:
            os.fsync(fd)
            os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
            done += 1
        except OSError:
            pass
        finally:
            os.close(fd)
    return done


def _fs_type(path: str) -> str:
    """File-system type of the mount holding path (/proc/mounts, longest prefix)."""
    best, fstype = "", "unknown"
    try:
        real = os.path.realpath(path)
        for line in Path("/proc/mounts").read_text().splitlines():
            f = line.split()
            if len(f) >= 3 and (real == f[1] or real.startswith(f[1].rstrip("/") + "/")) \
                    and len(f[1]) > len(best):
                best, fstype = f[1], f[2]
    except OSError:
        pass
    return fstype


def _resident_pages(paths) -> tuple[int, int]:
    """(resident, total) page-cache pages of these files, by mincore(2) over a
    read-only mapping of each."""
    import ctypes
    import mmap

    libc = ctypes.CDLL(None, use_errno=True)
    libc.mmap.restype = ctypes.c_void_p
    libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                          ctypes.c_int, ctypes.c_long]
    libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    libc.mincore.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    page = mmap.PAGESIZE
    res = tot = 0
    for p in paths:
        size = os.path.getsize(p)
        if size == 0:
            continue
        fd = os.open(p, os.O_RDONLY)
        try:
            addr = libc.mmap(None, size, mmap.PROT_READ, mmap.MAP_SHARED, fd, 0)
            if addr in (None, ctypes.c_void_p(-1).value):
                continue
            n = (size + page - 1) // page
            vec = (ctypes.c_ubyte * n)()
            if libc.mincore(addr, size, vec) == 0:
                res += sum(b & 1 for b in vec)
                tot += n
            libc.munmap(addr, size)
        finally:
            os.close(fd)
    return res, tot


def tt_config2_files(ctx, staged: list) -> dict:
    """BASELINE config 2 from files: each experiment's trace payload and long
    metric CSV go through load_experiment (native decoders) -> features() ->
    rank(), decode included in the timing."""
    def one(d, mc):
        return anomod.load_experiment(d, metrics=mc)

    one(*staged[0][:2])  # warm the page cache and the decoders
    t0 = time.perf_counter()
    t_dec = 0.0
    base = None
    hits = []
    spans = samples = 0
    for d, mc, fault in staged:
        a = time.perf_counter()
        e = one(d, mc)
        t_dec += time.perf_counter() - a
        f = anomod.features(e, ctx, baseline=base)
        if base is None:
            base = f
        else:
            hits.append(anomod.hit_at(anomod.rank(f, ctx=ctx), fault, 3))
        spans += e.spans.n_spans
        samples += e.metrics.S * e.metrics.T
    el = time.perf_counter() - t0
    # the same experiments again, each experiment's files dropped from the page
    # cache first (a collector's fresh files would be in it; a dataset read
    # back later would not)
    cold_dec, cold_tot, evicted = 0.0, 0.0, 0
    res_pages = tot_pages = 0
    fstype = _fs_type(str(staged[0][0])) if staged else "unknown"
    for d, mc, fault in staged:
        files = [str(x) for x in Path(d).rglob("*") if x.is_file()] + [mc]
        evicted += _evict_page_cache(files)
        r, t = _resident_pages(files)  # what the eviction actually left in memory
        res_pages += r
        tot_pages += t
        a = time.perf_counter()
        e = one(d, mc)
        cold_dec += time.perf_counter() - a
        anomod.features(e, ctx, baseline=base)
        cold_tot += time.perf_counter() - a
    sizes = [next(Path(d).glob("*.json")).stat().st_size for d, _, _ in staged]
    csv_sizes = [Path(mc).stat().st_size for _, mc, _ in staged]
    return {"experiments": len(staged), "spans": spans, "samples": samples, "seconds": el,
            "ms_per_experiment": el / len(staged) * 1e3, "decode_seconds": t_dec,
            "trace_json_mb_mean": float(np.mean(sizes)) / 1e6,
            "metric_csv_mb_mean": float(np.mean(csv_sizes)) / 1e6,
            "top3_hit_rate": float(np.mean(hits)),
            "cold_files": {"ms_per_experiment": cold_tot / len(staged) * 1e3,
                           "decode_ms_per_experiment": cold_dec / len(staged) * 1e3,
                           "files_fadvised": evicted, "staging_fs": fstype,
                           "resident_frac_after_evict": res_pages / tot_pages if tot_pages else None,
                           "valid": bool(tot_pages) and res_pages / tot_pages < 0.05,
                           "what": "load_experiment + features per experiment after "
                                   "fsync + posix_fadvise(DONTNEED) on its files; valid only when "
                                   "mincore shows < 5 % of their pages still resident (a tmpfs "
                                   "keeps them all: then this is a warm number)"},
            "note": "files in the dataset layout (collector payload JSON indent=2 + long metric "
                    "CSV) -> load_experiment (native decoders) -> features -> rank"}


def edge_leg(ctx, spans, reps: int, what: str) -> dict:
    """Edge-kernel time of a resident span set (hipEvents, ctx stream); the
    set's first aggregation (hints not learned yet) is reported as "cold"."""
    h0 = ctx.host_ms()
    t0 = time.perf_counter()
    ctx.edge_aggregate(spans, with_hist=False)
    cold = {"kernel_ms": ctx.stage_ms(L.STAGE_EDGE_AGG), "wall_ms": (time.perf_counter() - t0) * 1e3,
            "host_ms": host_paid(ctx, h0)}
    ms = []
    for _ in range(reps):
        ctx.edge_aggregate(spans, with_hist=False)
        ms.append(ctx.stage_ms(L.STAGE_EDGE_AGG))
    k = float(np.mean(ms))
    b = algorithmic_bytes(spans.n_spans, spans.n_traces)
    return {"what": what, "spans": spans.n_spans, "traces": spans.n_traces, "kernel_ms": k,
            "spans_per_s": spans.n_spans / (k * 1e-3), "bytes_per_launch": b,
            "achieved_GBps": b / (k * 1e-3) / 1e9, "frac": b / (k * 1e-3) / 1e9 / HBM_PEAK_GBPS,
            "cold": cold}


def group_bytes(info: dict, n: int, n_traces: int) -> int:
    """HBM bytes the grouping moves, by the path that ran (ctx.group_info())."""
    tiles = -(-n // 4096)
    if info["path"] == "bucket":
        # csrc/bucket.hip: level A counts read trace_hash (8 B) and the scatter
        # moves 32 B in + 32 B of records and 8 B of pairs out; with two levels
        # the level-B counts read the pairs (8 B) and level B moves them (8 + 8
        # B); the bucket kernel reads the pairs (8 B), gathers the records (32
        # B) and writes the SoA columns (32 B); trace starts: written, read,
        # written to trace_ptr (24 B/trace).  Tile counts (4 B per tile and
        # digit; level-B tiles are 16384 pairs): written, scanned (read twice,
        # written once), read by the scatter.
        T, two = info["bits"], info["levels"] == 2
        da = min(11, T) if not two else max(T - 11, min((T + 1) // 2, 9))
        db = T - da if two else 0
        b = 8 * n + 72 * n + 5 * 4 * tiles * (1 << da)
        if two:
            b += 8 * n + 16 * n + 5 * 4 * (-(-n // 16384)) * (1 << db)
        return b + 72 * n + 24 * n_traces
    if info["path"] == "join":
        # the same scatters; the join kernel reads the pairs (8 B), gathers
        # the records (32 B) and writes one 8-B edge record per span
        T, two = info["bits"], info["levels"] == 2
        da = min(11, T) if not two else max(T - 11, min((T + 1) // 2, 9))
        db = T - da if two else 0
        b = 8 * n + 72 * n + 5 * 4 * tiles * (1 << da)
        if two:
            b += 8 * n + 16 * n + 5 * 4 * (-(-n // 16384)) * (1 << db)
        return b + 48 * n
    # csrc/group.hip (LSD): the first pass's tile counts read trace_hash, later
    # passes' the 1-B digits the previous pass wrote (written + read: 2 B);
    # each radix pass reads and writes 32 B (records, the last one the SoA
    # columns); the bucket-list and trace_ptr scans read the grouped hashes;
    # trace_ptr writes 8 B/trace
    P = info["levels"]
    return 8 * n + 2 * (P - 1) * n + 64 * P * n + 16 * n + 8 * n_traces


def host_paid(ctx, before: dict) -> dict:
    """The host slots (anomod_ctx_host_ms) a call paid since `before`: the
    one-off setup steps (workspace allocations, upload pipeline) and the
    grouping stage's host wall, in ms."""
    return {k: round(v[0], 3) for k, v in ctx.host_ms().items() if v[1] != before[k][1]}


def ungrouped_leg(ctx, inter, n_traces: int, allsum) -> dict:
    """Grouping + edge aggregation of an ungrouped resident set (n_traces:
    the traces it holds, all non-empty)."""
    h0 = ctx.host_ms()
    t0 = time.perf_counter()
    ctx.edge_aggregate(inter, with_hist=False)
    cold = {"wall_ms": (time.perf_counter() - t0) * 1e3, "group_ms": ctx.stage_ms(L.STAGE_GROUP),
            "edge_ms": ctx.stage_ms(L.STAGE_EDGE_AGG), "host_ms": host_paid(ctx, h0)}
    g, e, wall = [], [], []
    for _ in range(3):
        t0 = time.perf_counter()
        ctx.edge_aggregate(inter, with_hist=False)
        wall.append(time.perf_counter() - t0)
        g.append(ctx.stage_ms(L.STAGE_GROUP))
        e.append(ctx.stage_ms(L.STAGE_EDGE_AGG))
    n, info = inter.n_spans, ctx.group_info()
    gbytes = group_bytes(info, n, n_traces)
    g_ms, e_ms = float(np.mean(g)), float(np.mean(e))
    return {"what": "SN spans of every 4096 consecutive traces interleaved (ES start_time "
                    "order); step = device grouping + edge aggregation (group_path join: "
                    "bucket scatters + per-bucket parent hash join writing edge records, "
                    "group_ms; the table from the records, edge_ms)",
            "spans": n, "traces": n_traces, "group_path": info,
            "spans_per_s": allsum(n / float(np.mean(wall))), "step_ms": float(np.mean(wall)) * 1e3,
            "group_ms": g_ms, "edge_ms": e_ms,
            "group_bytes": gbytes, "group_GBps": gbytes / (g_ms * 1e-3) / 1e9,
            "group_frac": gbytes / (g_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
            # against what grouping must move at least: read and write each
            # 32-B span once (64 B/span); the whole step against its 32 B/span in
            "group_algo_frac": 64 * n / (g_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
            "step_algo_frac": 32 * n / (float(np.mean(wall))) / 1e9 / HBM_PEAK_GBPS,
            "cold": cold}


def load_traffic(n_spans: int) -> tuple[float | None, dict | None]:
    """HBM bytes per launch from the committed PMC profile of this workload,
    and where they came from (file, round, the commit the profiled library was
    built from, kernel, correction): the value is not measured in this run."""
    p = ROOT / "profiles" / "edge_agg_pmc.json"
    try:
        d = json.loads(p.read_text())
        if int(d["n_spans"]) == n_spans:
            src = {"file": str(p.relative_to(ROOT)), "round": d.get("round"),
                   "commit": d.get("commit"), "kernel": d.get("kernel"),
                   "correction": d.get("correction"),
                   "measured_in_this_run": False}
            return float(d["hbm_bytes_per_launch"]), src
    except Exception:
        pass
    return None, None


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--traces-per-gpu", type=int, default=1 << 27)
    ap.add_argument("--seed", type=int, default=20251103)
    ap.add_argument("--cpu-traces", type=int, default=1 << 21)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--leg-cpu-seconds", type=float, default=6.0,
                    help="CPU-baseline time per extra leg (trace structure, grouping, EWMA, "
                         "PageRank)")
    ap.add_argument("--host-comm", action="store_true",
                    help="N > 1 rehearsal on one device: the ranks merge through libanomod's "
                         "host collective transport over the HostGroup instead of RCCL")
    ap.add_argument("--no-extras", action="store_true", help="headline line only")
    ap.add_argument("--legs", default=",".join(LEGS),
                    help="extra legs to run (comma list of " + ", ".join(LEGS) + ")")
    ap.add_argument("--ppr-nodes", type=int, default=100_000)
    ap.add_argument("--ppr-iters", type=int, default=100)
    ap.add_argument("--ewma-series", type=int, default=100_000)
    ap.add_argument("--ewma-steps", type=int, default=131040, help="steps per chunk")
    ap.add_argument("--ewma-chunks", type=int, default=8)
    args = ap.parse_args()
    legs = set() if args.no_extras else {x for x in args.legs.split(",") if x}
    unknown = legs - set(LEGS)
    if unknown:
        ap.error(f"unknown legs {sorted(unknown)}")

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    group = None
    if world > 1:
        # host-side control plane: a stdlib TCP group (no torch.distributed):
        # the RCCL unique id, barriers and the scalar max/sum of the timings
        from anomod import dist

        group = dist.HostGroup(rank, world)
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)

    def barrier():
        if group is not None:
            group.barrier()

    def allmax(v: float) -> float:
        return v if group is None else group.allreduce_scalar(v, L.OP_MAX)

    def allsum(v: float) -> float:
        return v if group is None else group.allreduce_scalar(v, L.OP_SUM)

    staged = None
    if "tt_config2_files" in legs and world == 1:
        # staged before the GPU is touched (the pool forks)
        import tempfile

        stage_root = tempfile.mkdtemp(prefix="anomod_tt_files_")
        t_stage = time.perf_counter()
        staged = stage_tt_files(stage_root)
        t_stage = time.perf_counter() - t_stage

    ctx = anomod.Context(0 if args.host_comm else local)
    transport = "none"
    if world > 1:
        if args.host_comm:  # ranks sharing one GPU (RCCL refuses): same calls, host transport
            dist.attach_host(ctx, group)
            transport = "host (HostGroup, one device)"
        else:  # RCCL; the host transport only if RCCL refuses on every rank (said in the line)
            transport = dist.attach(ctx, dist.RankInfo(rank, world, local), group)
    coll = "RCCL" if transport == "rccl" else "host"
    cpu_legs = rank == 0 and world == 1 and not args.no_cpu_baseline

    spec = anomod.SynthSpec("SN", seed=args.seed, p_orphan_ppm=100)
    spans = ctx.generate(spec, args.traces_per_gpu, shard=rank)  # this rank's traces, in HBM

    cold = None
    for w in range(args.warmup):
        t0 = time.perf_counter()
        ctx.edge_aggregate(spans, with_hist=False)
        if w == 0:  # the set's first aggregation: histogram form not known yet
            cold = {"kernel_ms": ctx.stage_ms(L.STAGE_EDGE_AGG),
                    "wall_ms": (time.perf_counter() - t0) * 1e3}
    ctx.synchronize()
    barrier()
    ctx.synchronize()
    kernel_ms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        table = ctx.edge_aggregate(spans, with_hist=False)
        kernel_ms.append(ctx.stage_ms(L.STAGE_EDGE_AGG))
    ctx.synchronize()
    barrier()
    el = allmax(time.perf_counter() - t0)
    total_spans = allsum(float(spans.n_spans))
    assert int(table.count.sum()) == (int(total_spans) if world > 1 else spans.n_spans)

    k_ms = float(np.mean(kernel_ms))
    bytes_launch = algorithmic_bytes(spans.n_spans, spans.n_traces)
    achieved = bytes_launch / (k_ms * 1e-3) / 1e9
    traffic, traffic_src = load_traffic(spans.n_spans)
    result = {
        "metric": METRIC,
        "value": total_spans * args.steps / el,
        "unit": "spans/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (DeathStarBench SocialNetwork topology, generated in HBM)",
        "config": {
            "workload": "config 3 shape: synthetic SN spans grouped by trace, "
                        f"{args.traces_per_gpu} traces (~{spans.n_spans / 1e9:.2f}e9 spans) "
                        "per GPU, edge table + 896-bin histograms + p50/p99 per step",
            "spans_per_gpu": spans.n_spans, "traces_per_gpu": spans.n_traces,
            "services": len(spans.services), "hist_bins": L.HIST_BINS,
            "parallelism": f"dp{world} (traceId shards)" + (f" + {coll} all-reduce" if world > 1
                                                            else ""),
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic, "traffic_source": traffic_src,
            "kernel": "edge_agg_kernel<lds_hist,lds_stats>", "kernel_ms": k_ms,
            "bytes_per_launch": bytes_launch,
        },
        "cold": cold,
    }
    if world > 1:
        result["transport"] = transport
    if "general_scan" in legs:
        # --- the same spans without the generator's unique-id declaration
        # (ANOMOD_UNIQUE_SCAN=0): the first-match forward parent scan every
        # set takes when nothing is known about duplicated ids
        os.environ["ANOMOD_UNIQUE_SCAN"] = "0"
        try:
            result["sn_general_scan"] = edge_leg(ctx, spans, 3, "edge kernel, first-match forward "
                                                 "scan (ids not declared unique)")
        finally:
            del os.environ["ANOMOD_UNIQUE_SCAN"]
    if "trace_structure" in legs:
        # --- trace structure on the same resident spans:
        # reads 20 B/span + 8 B/trace, writes 13 B/span + 12 B/trace
        ctx.trace_structure(spans, download=False)
        ts_ms = []
        for _ in range(3):
            ctx.trace_structure(spans, download=False)
            ts_ms.append(ctx.stage_ms(L.STAGE_TRACE_STRUCT))
        t_ms = float(np.mean(ts_ms))
        ts_bytes = 33 * spans.n_spans + 20 * spans.n_traces
        result["trace_structure"] = {
            "spans_per_s": allsum(spans.n_spans / (t_ms * 1e-3)), "kernel_ms": t_ms,
            "bytes_per_launch": ts_bytes, "achieved_GBps": ts_bytes / (t_ms * 1e-3) / 1e9,
            "frac": ts_bytes / (t_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS}
        if cpu_legs:
            result["trace_structure"]["cpu_baseline"] = cpu_trace_structure(
                spec, 1 << 19, args.leg_cpu_seconds)
    if "exact_quantiles" in legs:
        # --- §8a a11 cross-check: exact per-edge order statistics (edge keys
        # + one radix sort) against the histogram quantiles of the headline
        # table: the bin-midpoint error the histogram costs
        t0 = time.perf_counter()
        ex, cnt = ctx.edge_quantiles_exact(spans, (50, 99))
        q_s = time.perf_counter() - t0
        ok = cnt > 0
        rel = {}
        for k, name in ((0, "p50_us"), (1, "p99_us")):
            h = getattr(table, name)[ok]
            x = ex[ok, k]
            r = np.abs(h - x) / np.maximum(x, 1.0)
            rel[name] = {"max_rel_err": float(r.max()), "mean_rel_err": float(r.mean())}
        result["exact_quantiles"] = {
            "what": "exact x[int(c*q)] per edge vs the 896-bin histogram midpoints",
            "edges": int(ok.sum()), "seconds": q_s, **rel}
    if "in_trace_shuffled" in legs:
        # --- the same spans with every trace's spans in a random order (the
        # parent scan can no longer rely on parents sitting early)
        intra = ctx.shuffle(spans, seed=args.seed + 1, window_traces=0)
        result["sn_in_trace_shuffled"] = edge_leg(ctx, intra, 3, "edge kernel on SN spans "
                                                  "shuffled inside every trace")
        intra.free()
    if "ungrouped" in legs:
        # --- ungrouped input (north_star (2)): the spans of every 4096
        # consecutive traces interleaved in a random order, as the ES path
        # pulls hits sorted by start_time across concurrent traces
        # (enhanced_trace_collector.py:80-90); a step = device grouping
        # (segmented radix sort) + edge aggregation
        h0 = ctx.host_ms()
        t0 = time.perf_counter()
        inter = ctx.shuffle(spans, seed=args.seed + 2, window_traces=4096)
        prep = {"wall_ms": (time.perf_counter() - t0) * 1e3, "host_ms": host_paid(ctx, h0)}
        result["ungrouped"] = ungrouped_leg(ctx, inter, spans.n_traces, allsum)
        # making the interleaved set (not timed: input preparation) reserves the
        # context's grouping workspace for it (anomod_ctx_reserve_grouping)
        result["ungrouped"]["set_prep"] = prep
        inter.free()
        if cpu_legs:
            result["ungrouped"]["cpu_baseline"] = cpu_group(spec, 1 << 18, args.leg_cpu_seconds)
    spans.free()
    if "tt_width" in legs:
        # --- TrainTicket width (BASELINE config 2 topology, 46 services:
        # E = 2208 edges) at 2^27 traces (~3.1e9 spans, one launch)
        tt = ctx.generate(anomod.SynthSpec("TT", seed=args.seed, p_orphan_ppm=100),
                          args.traces_per_gpu, shard=rank)
        result["tt_width"] = edge_leg(ctx, tt, 3, "edge kernel on synthetic TrainTicket spans")
        tt.free()
    if "long_traces" in legs:
        # --- trace length / depth stress (SynthSpec LONG: SN services, traces
        # of 16..4000 spans, 30 % of the spans in traces longer than a wave
        # chunk -> the workgroup-per-trace pass), 2^23 traces (~4.4e8 spans)
        lt = ctx.generate(anomod.SynthSpec("LONG", seed=args.seed, p_orphan_ppm=100),
                          max(1, args.traces_per_gpu // 16), shard=rank)
        result["long_traces"] = edge_leg(ctx, lt, 3, "edge kernel on LONG spans (traces of "
                                         "16..4000 spans; > 256 via the workgroup-per-trace pass)")
        lt.free()
        # the product path's first call: a host LONG set uploaded per call
        # (Context.edge_aggregate / features()); its learned hints stay on the
        # host SpanSet, so the second call starts from them
        lh = ctx.generate(anomod.SynthSpec("LONG", seed=args.seed + 3, p_orphan_ppm=100),
                          1 << 20, shard=rank)
        host = lh.download()
        lh.free()
        calls = []
        for _ in range(3):
            h0 = ctx.host_ms()
            t0 = time.perf_counter()
            ctx.edge_aggregate(host, with_hist=True)
            calls.append({"wall_ms": (time.perf_counter() - t0) * 1e3,
                          "kernel_ms": ctx.stage_ms(L.STAGE_EDGE_AGG),
                          "host_ms": host_paid(ctx, h0)})
        result["long_traces"]["host_set_calls"] = {
            "spans": host.n_spans, "what": "Context.edge_aggregate(host SpanSet): upload + "
                                           "aggregate + download, first call then two more",
            "calls": calls}
        del host

    if "pagerank" in legs:
        # --- PageRank RCA: replicas (one graph + personalization per GPU)
        g = anomod.DeviceGraph(ctx, synthetic=(args.ppr_nodes, 10, 11 + rank))
        p = np.random.default_rng(rank).random(g.N)
        t0 = time.perf_counter()
        g.pagerank(p, iters=args.ppr_iters)  # capture + warm
        ppr_cold = (time.perf_counter() - t0) * 1e3
        reps = 10
        barrier()
        t0 = time.perf_counter()
        pr_ms = []
        for _ in range(reps):
            g.pagerank(p, iters=args.ppr_iters)
            pr_ms.append(ctx.stage_ms(L.STAGE_PAGERANK))
        pel = allmax(time.perf_counter() - t0)
        ppr_bytes = 4 * (g.N + 1) + 8 * g.nnz + 16 * g.N  # in_ptr + (col,w) + x gather/write
        result["pagerank"] = {
            "iters_per_s": world * reps * args.ppr_iters / pel,
            "cold_solve_ms": None,
            "device_iters_per_s_per_gpu": args.ppr_iters / (np.mean(pr_ms) * 1e-3),
            "nodes": g.N, "edges": g.nnz, "iters_per_solve": args.ppr_iters,
            "mode": "replicas (independent personalization per GPU, no collective)",
            "bytes_per_iter": ppr_bytes,
            "achieved_GBps": ppr_bytes * args.ppr_iters / (np.mean(pr_ms) * 1e-3) / 1e9,
        }
        result["pagerank"]["cold_solve_ms"] = ppr_cold
        if cpu_legs:
            result["pagerank"]["cpu_baseline"] = cpu_pagerank(args.ppr_nodes, args.ppr_iters, 11,
                                                              args.leg_cpu_seconds)
        # row-sharded solve (SURVEY §8e "sharded" series): one vector over all
        # ranks, whole 256-row blocks per rank, one grouped RCCL exchange per
        # iteration (u64 partial sums + in-place all-gather of x); at N=1 the
        # same loop without a communicator
        gs = anomod.DeviceGraph(ctx, synthetic=(args.ppr_nodes, 10, 11))  # same graph everywhere
        ps = np.random.default_rng(7).random(gs.N)  # and the same vector
        gs.pagerank_sharded(ps, iters=args.ppr_iters)
        sh_ms = []
        for _ in range(3):
            barrier()
            gs.pagerank_sharded(ps, iters=args.ppr_iters)
            sh_ms.append(ctx.stage_ms(L.STAGE_PAGERANK))
        gs.free()
        s_ms = allmax(float(np.mean(sh_ms)))
        result["pagerank"]["sharded"] = {
            "iters_per_s": args.ppr_iters / (s_ms * 1e-3), "shards": world,
            "us_per_iter": s_ms * 1e3 / args.ppr_iters,
            "mode": f"row-sharded, per-iteration launches + {coll} all-reduce/all-gather"
                    if world > 1 else "row-sharded path, 1 shard (per-iteration launches)"}
        # batched personalizations (one per fault hypothesis)
        # (one persistent launch per batch: K vectors per grid barrier; K = 16
        # in workgroups of two 256-row blocks)
        for kb, key in ((8, "batched"), (16, "batched_k16")):
            Pb = np.random.default_rng(100 + rank + kb).random((kb, g.N))
            g.pagerank_batch(Pb, iters=args.ppr_iters)
            bt, bw = [], []
            barrier()
            t0 = time.perf_counter()
            for _ in range(3):
                t1 = time.perf_counter()
                g.pagerank_batch(Pb, iters=args.ppr_iters)
                bw.append(round((time.perf_counter() - t1) * 1e3, 3))
                bt.append(ctx.stage_ms(L.STAGE_PAGERANK))
            bwall = allmax(time.perf_counter() - t0)
            b_ms = float(np.mean(bt))
            result["pagerank"][key] = {
                "vectors": kb, "path": g.last_solve()[0],
                "vector_iters_per_s": world * 3 * kb * args.ppr_iters / bwall,
                "vector_iters_per_s_per_gpu": kb * args.ppr_iters / (b_ms * 1e-3),
                "iters_per_s_per_gpu": args.ppr_iters / (b_ms * 1e-3),
                "us_per_batched_iter": b_ms * 1e3 / args.ppr_iters,
                "wall_ms_per_batch": bw, "last_solve": list(g.last_solve()),
                "what": f"solved vector-iterations/s (wall, all ranks) of {kb}-vector batches; "
                        f"per-GPU device rates from the kernel time"}
        g.free()
    if "ewma" in legs:
        # --- EWMA/z, BASELINE config 4 at its size: S = 10^5 series x ~10^6
        # steps (8 chunks of 131 040 steps = 52 GB each: X is 400 GB, more
        # than HBM).  Each chunk is generated in HBM (fill_synthetic(t0),
        # outside the timing) and scored with the (m, v, n) state carried
        # from the previous chunk; the kernel times of all chunks are summed.
        W = 60
        ser = anomod.DeviceSeries(ctx, args.ewma_steps, args.ewma_series)
        ser.fill_synthetic(7 + rank, 0)
        t0 = time.perf_counter()
        ser.ewma_z(2 / (W + 1), W, download=False)  # warm
        ew_cold = {"wall_ms": (time.perf_counter() - t0) * 1e3,
                   "kernel_ms": ctx.stage_ms(L.STAGE_EWMA)}
        ser.reset_state()
        ew = []
        for c in range(args.ewma_chunks):
            ser.fill_synthetic(7 + rank, c * args.ewma_steps)
            ser.ewma_z(2 / (W + 1), W, download=False)
            ew.append(ctx.stage_ms(L.STAGE_EWMA))
        e_ms = float(np.sum(ew))
        samples = args.ewma_chunks * args.ewma_steps * args.ewma_series
        # 4 B/sample read + 4/W B/sample written + per-chunk state (m, v f64 + n u32, r+w)
        e_bytes = 4 * samples + 4 * samples // W + 40 * args.ewma_series * args.ewma_chunks
        result["ewma"] = {
            "samples_per_s": allsum(samples / (e_ms * 1e-3)),
            "T": args.ewma_chunks * args.ewma_steps, "S": args.ewma_series, "W": W,
            "chunks": args.ewma_chunks, "steps_per_chunk": args.ewma_steps,
            "kernel_ms": e_ms, "chunk_ms": [round(x, 4) for x in ew],
            "achieved_GBps": e_bytes / (e_ms * 1e-3) / 1e9,
            "frac": e_bytes / (e_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
            "note": "config 4 at size: chunks generated in HBM outside the timing, state carried",
            "cold_chunk": ew_cold,
        }
        ser.free()
        if cpu_legs:
            result["ewma"]["cpu_baseline"] = cpu_ewma(args.ewma_steps // 8 // W * W, 1000, W,
                                                      args.leg_cpu_seconds)

    if "tt_config2" in legs and world == 1:
        result["tt_config2"] = tt_config2(ctx)
    if staged is not None:
        result["tt_config2_files"] = tt_config2_files(ctx, staged)
        result["tt_config2_files"]["staging_seconds"] = t_stage
        import shutil

        shutil.rmtree(stage_root, ignore_errors=True)

    if cpu_legs:
        result["cpu_baseline"] = cpu_baseline(spec, args.cpu_traces, args.cpu_seconds)

    ctx.close()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if group is not None:
        group.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
