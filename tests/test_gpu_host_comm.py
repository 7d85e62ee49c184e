"""GPU: libanomod's multi-rank path with two ranks on one device, through the
host collective transport (anomod_ctx_attach_host_comm, driven by gloo via
anomod.dist.attach_host over a stdlib TCP HostGroup) — RCCL refuses two ranks on a GPU, so this is how
the 1-GPU box runs the collective sequence with nranks = 2:

* edge table: traceId-hash shards, status agreement, u64 sum /
  u32 min / u32 max merge -> every rank holds the oracle's unsharded table;
* status agreement: one rank's invalid call fails BOTH ranks (no rank waits
  in the merge), and the transport is dropped afterwards on neither;
* row-sharded PageRank: per-iteration u64 all-reduces + x all-gather -> the
  vector equals the unsharded solve bit for bit, in fixed and tolerance mode;
* ungrouped spans: device grouping per shard, then the same merge.
"""
import os
import socket
import subprocess
import sys
import textwrap

import numpy as np
import pytest

import anomod
from oracle import native

from conftest import PKG_DIR, ROOT
from test_gpu_edge import assert_table_equal

pytestmark = pytest.mark.gpu

_WORKER = textwrap.dedent("""
    import os, sys
    sys.path[:0] = [{pkg!r}, {root!r}]
    import numpy as np
    import anomod
    from anomod import dist
    info = dist.rank_from_env()
    grp = dist.HostGroup(info.rank, info.world)
    out = {{}}
    sp = anomod.synth_generate_host(anomod.SynthSpec("SN", seed=9, p_orphan_ppm=3000), 30000)
    part = dist.shard_spans(sp, info)
    with anomod.Context(0) as c:
        dist.attach_host(c, grp)
        assert c.comm_info() == (2, info.rank)
        t = c.edge_aggregate(part)
        for k in ("count", "errors", "sum_us", "min_us", "max_us", "hist", "p50_us", "p99_us"):
            out[k] = getattr(t, k)
        out["n_part"] = part.n_spans
        # status agreement: rank 1 asks for too few services -> both ranks fail
        bad = part if info.rank == 0 else anomod.SpanSet(part.services[:2], part.trace_ptr,
            part.trace_hash, part.span_id, part.parent_span_id, part.svc, part.flags, part.dur_us)
        try:
            c.edge_aggregate(bad)
            out["agree_err"] = ""
        except anomod.AnomodError as e:
            out["agree_err"] = str(e)
        # the transport survives an agreed failure: a second merge works
        t2 = c.edge_aggregate(part)
        out["count2"] = t2.count
        # ungrouped spans (arrival order interleaved) -> grouping on device, same merge
        dev = c.upload(part)
        ug = c.shuffle(dev, seed=3, window_traces=64)
        t3 = c.edge_aggregate(ug)
        out["count3"] = t3.count
        out["hist3"] = t3.hist
        ug.free()
        dev.free()
        # row-sharded PageRank over the two ranks vs this rank's unsharded solve
        # (default path: the persistent solve beside the other rank's process,
        # rerun per launch if a workgroup cannot become resident)
        g = anomod.DeviceGraph(c, synthetic=(30000, 8, 6))
        p = np.random.default_rng(1).random(g.N)
        for iters, tol in ((37, 0.0), (1000, 1e-10)):
            xs, ds = g.pagerank_sharded(p, iters=iters, tol=tol)
            x, d = g.pagerank(p, iters=iters, tol=tol)
            out[f"ppr_eq_{{iters}}"] = int(np.array_equal(xs, x) and ds == d)
            out[f"ppr_path_{{iters}}"] = g.last_solve()[0]
        g.free()
    np.savez(os.path.join({out!r}, f"rank{{info.rank}}.npz"), **out)
    grp.barrier()
    grp.close()
    assert "torch" not in sys.modules
""")


def test_two_ranks_host_transport(tmp_path):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    script = tmp_path / "worker.py"
    script.write_text(_WORKER.format(pkg=str(PKG_DIR), root=str(ROOT), out=str(tmp_path)))
    procs = []
    for r in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                   WORLD_SIZE="2", LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      start_new_session=True))
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=100)[0].decode(errors="replace"))
        except subprocess.TimeoutExpired:
            for q in procs:
                if q.poll() is None:
                    os.killpg(q.pid, 9)
            pytest.fail("two-rank host-transport run timed out")
    assert all(p.returncode == 0 for p in procs), "\n".join(outs)[-3000:]
    sp = anomod.synth_generate_host(anomod.SynthSpec("SN", seed=9, p_orphan_ppm=3000), 30000)
    ref = native.edge_aggregate(sp, len(sp.services))
    r0, r1 = (np.load(tmp_path / f"rank{r}.npz") for r in range(2))
    assert int(r0["n_part"]) + int(r1["n_part"]) == sp.n_spans
    assert 0 < int(r0["n_part"]) < sp.n_spans
    for r in (r0, r1):
        got = anomod.EdgeTable(services=sp.services, **{k: r[k] for k in (
            "count", "errors", "sum_us", "min_us", "max_us", "hist", "p50_us", "p99_us")})
        assert_table_equal(got, ref)
        np.testing.assert_array_equal(r["count2"], ref["count"])
        np.testing.assert_array_equal(r["count3"], ref["count"])
        np.testing.assert_array_equal(r["hist3"], ref["hist"])
        assert r["ppr_eq_37"] == 1 and r["ppr_eq_1000"] == 1
    assert "n_services" in str(r1["agree_err"])     # the failing rank's own reason
    assert str(r0["agree_err"]) != ""                 # its peer failed with it


@pytest.mark.parametrize("mode", ["host_comm", "fallback"])
def test_bench_two_ranks_host_comm(tmp_path, mode):
    """bench.py's N > 1 code — HostGroup rendezvous, per-step edge-table
    merge, barriers, allmax / allsum weak-scaling accounting — run for real
    at world 2 on one MI355X through the host transport, with every leg the
    driver's N > 1 runs (each rank must enter the same collectives in the
    same order, or the run hangs), at small sizes.  host_comm: --host-comm;
    fallback: no flag and both ranks on device 0 (LOCAL_RANK 0), so RCCL
    refuses on both and dist.attach takes the host transport, saying so in
    the line.  bench.py itself asserts the merged count.sum() equals the
    spans of both shards."""
    import json

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                   WORLD_SIZE="2", LOCAL_RANK=str(r if mode == "host_comm" else 0),
                   ANOMOD_RDZV_DIR=str(tmp_path))
        procs.append(subprocess.Popen(
            [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "3",
             "--warmup", "1", "--traces-per-gpu", "30000", "--ppr-nodes", "20000",
             "--ppr-iters", "20", "--ewma-series", "2000", "--ewma-steps", "1920",
             "--ewma-chunks", "2", "--no-cpu-baseline"]
            + (["--host-comm"] if mode == "host_comm" else []),
            env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, start_new_session=True))
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=150)
            outs.append((o.decode(errors="replace"), e.decode(errors="replace")))
        except subprocess.TimeoutExpired:
            for q in procs:
                if q.poll() is None:
                    os.killpg(q.pid, 9)
            pytest.fail("two-rank bench run timed out")
    assert all(p.returncode == 0 for p in procs), outs
    line = json.loads(outs[0][0].strip().splitlines()[-1])
    assert outs[1][0].strip() == ""  # only rank 0 prints
    assert line["n_gpus"] == 2 and line["transport"].startswith("host")
    if mode == "fallback":
        assert line["transport"].startswith("host (RCCL refused")
        assert "host all-reduce" in line["config"]["parallelism"]
    for leg in ("sn_general_scan", "trace_structure", "exact_quantiles", "sn_in_trace_shuffled",
                "ungrouped", "tt_width", "long_traces", "pagerank", "ewma"):
        assert leg in line, leg
    n0 = anomod.synth_generate_host(anomod.SynthSpec("SN", seed=20251103, p_orphan_ppm=100),
                                    30000, shard=0).n_spans
    n1 = anomod.synth_generate_host(anomod.SynthSpec("SN", seed=20251103, p_orphan_ppm=100),
                                    30000, shard=1).n_spans
    assert line["config"]["spans_per_gpu"] == n0
    assert line["value"] == pytest.approx((n0 + n1) * 3 / (line["ms_per_step"] * 3e-3))
    assert line["ungrouped"]["spans"] == n0
    assert line["pagerank"]["sharded"]["shards"] == 2
