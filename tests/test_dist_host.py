"""Multi-rank host plumbing on CPU without torch: anomod.dist.HostGroup (a
stdlib TCP group) carries the RCCL unique id, barriers, scalar reductions and
libanomod's host collective transport.  World 2 and 3 as separate processes:

* broadcast / barrier / all-reduce (u64 sum wrapping mod 2^64, u32 min / max,
  f64) / all-gather give every rank the same bytes;
* traceId-hash shards + the HostGroup integer merge reproduce the unsharded
  edge table of the CPU oracle bit for bit (the per-rank partial tables come
  from the oracle: no GPU here; the sharding is the product's);
* importing anomod / anomod.dist and forming a group never imports torch.
"""
import json
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

from conftest import PKG_DIR, ROOT

_WORKER = textwrap.dedent("""
    import json, os, sys
    sys.path[:0] = [{pkg!r}, {root!r}]
    import numpy as np
    import anomod
    from anomod import dist, _lib as L
    from oracle import native
    info = dist.rank_from_env()
    out = {{}}
    with dist.HostGroup(info.rank, info.world, key={key!r}, rdzv_dir={rdzv!r}, timeout_s=60) as g:
        out["uid"] = g.broadcast(bytes(range(128)) if info.rank == 0 else None).hex()
        g.barrier()
        a = np.array([2**64 - 1 - info.rank, 5 + info.rank], dtype=np.uint64)
        g.allreduce(a, L.OP_SUM)
        out["u64sum"] = [int(x) for x in a]
        b = np.array([4000000000 - info.rank, 7 * info.rank], dtype=np.uint32)
        c = b.copy()
        g.allreduce(b, L.OP_MIN)
        g.allreduce(c, L.OP_MAX)
        out["u32min"], out["u32max"] = [int(x) for x in b], [int(x) for x in c]
        out["f64"] = g.allreduce_scalar(0.5 * (info.rank + 1), L.OP_SUM)
        buf = np.zeros(3 * info.world, dtype=np.uint8)
        buf[3 * info.rank:3 * info.rank + 3] = 10 * info.rank + np.arange(3)
        g.allgather(buf, 3)
        out["gather"] = buf.tolist()
        # traceId-hash shard + integer merge == the unsharded table
        spans = anomod.synth_generate_host(anomod.SynthSpec("SN", seed=77, p_orphan_ppm=2000), 6000)
        part = dist.shard_spans(spans, info)
        tab = native.edge_aggregate(part, len(spans.services))
        for k, op in (("count", L.OP_SUM), ("errors", L.OP_SUM), ("sum_us", L.OP_SUM),
                      ("hist", L.OP_SUM), ("min_us", L.OP_MIN), ("max_us", L.OP_MAX)):
            g.allreduce(tab[k], op)
        out["n_part"] = part.n_spans
        np.savez(os.path.join({out!r}, f"tab{{info.rank}}.npz"), **tab)
    out["torch_loaded"] = "torch" in sys.modules
    with open(os.path.join({out!r}, f"rank{{info.rank}}.json"), "w") as f:
        json.dump(out, f)
""")


def _run(tmp_path, world: int):
    script = tmp_path / "worker.py"
    key = f"t{os.getpid()}-{world}"
    script.write_text(_WORKER.format(pkg=str(PKG_DIR), root=str(ROOT), out=str(tmp_path),
                                     key=key, rdzv=str(tmp_path)))
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=120)[0].decode(errors="replace"))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            pytest.fail("host-group run timed out")
    assert all(p.returncode == 0 for p in procs), "\n".join(outs)[-3000:]
    return [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(world)]


@pytest.mark.parametrize("world", [2, 3])
def test_host_group_collectives(tmp_path, world):
    res = _run(tmp_path, world)
    ranks = range(world)
    for r in res:
        assert bytes.fromhex(r["uid"]) == bytes(range(128))
        assert r["u64sum"] == [sum(2**64 - 1 - k for k in ranks) % 2**64, sum(5 + k for k in ranks)]
        assert r["u32min"] == [4000000000 - (world - 1), 0]
        assert r["u32max"] == [4000000000, 7 * (world - 1)]
        assert r["f64"] == sum(0.5 * (k + 1) for k in ranks)
        assert r["gather"] == [10 * k + j for k in ranks for j in range(3)]
        assert r["torch_loaded"] is False

    import anomod
    from oracle import native

    spans = anomod.synth_generate_host(anomod.SynthSpec("SN", seed=77, p_orphan_ppm=2000), 6000)
    whole = native.edge_aggregate(spans)
    assert sum(r["n_part"] for r in res) == spans.n_spans
    assert all(0 < r["n_part"] < spans.n_spans for r in res)
    for k in ranks:
        tab = np.load(tmp_path / f"tab{k}.npz")
        for key in ("count", "errors", "sum_us", "hist", "min_us", "max_us"):
            np.testing.assert_array_equal(tab[key], whole[key], err_msg=key)


def test_import_without_torch():
    code = ("import sys; sys.path[:0] = [%r, %r]; import anomod, anomod.dist; "
            "g = anomod.dist.HostGroup(0, 1); g.barrier(); "
            "print('torch' in sys.modules)") % (str(PKG_DIR), str(ROOT))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "False"


def test_rendezvous_survives_stray_clients(tmp_path):
    """Rank 0 drops clients that close at once, send garbage or a bad hello
    (a stale rank of an earlier run) instead of aborting the rendezvous; the
    real ranks still form the group (threads of one process here)."""
    import json as _json
    import socket
    import struct
    import threading
    import time

    from anomod import dist

    key, res, errs = f"stray{os.getpid()}", {}, []

    def rank(r):
        try:
            with dist.HostGroup(r, 2, key=key, rdzv_dir=str(tmp_path), timeout_s=30) as g:
                res[r] = g.allreduce_scalar(r + 1.0)
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    t0 = threading.Thread(target=rank, args=(0,))
    t0.start()
    path = tmp_path / f"anomod-rdzv-{key}.json"
    deadline = time.monotonic() + 20
    while not path.exists() and time.monotonic() < deadline:
        time.sleep(0.02)
    info = _json.loads(path.read_text())
    addr = (info["addr"], info["port"])
    socket.create_connection(addr).close()                      # closes at once
    s = socket.create_connection(addr)
    s.sendall(struct.pack("<Q", 3) + b"xyz")                    # too short a hello
    s.close()
    s = socket.create_connection(addr)
    s.sendall(struct.pack("<Q", 12) + b"ANMD" + struct.pack("<ii", 5, 9))  # stale world
    t1 = threading.Thread(target=rank, args=(1,))
    t1.start()
    t0.join(60)
    t1.join(60)
    s.close()
    assert not errs, errs
    assert res == {0: 3.0, 1: 3.0}


def test_silent_peer_times_out(tmp_path):
    """A rank that stops answering without closing its socket (stuck in a GPU
    call, a lost host) makes the others raise TimeoutError after the
    collective timeout instead of waiting forever; keepalive is on every
    peer link (threads of one process here; rank 1 forms the group, then
    never enters the barrier)."""
    import socket
    import threading

    from anomod import dist

    key, errs, formed, release = f"silent{os.getpid()}", {}, threading.Event(), threading.Event()
    groups, keepalive = {}, {}

    def rank(r):
        try:
            g = dist.HostGroup(r, 2, key=key, rdzv_dir=str(tmp_path), timeout_s=30,
                               coll_timeout_s=1.5)
            groups[r] = g
            if r == 1:
                formed.set()
                release.wait(30)  # silent: socket open, no collective
            else:
                formed.wait(30)
                keepalive[r] = g._peers[0].getsockopt(socket.SOL_SOCKET, socket.SO_KEEPALIVE)
                g.barrier()
        except Exception as e:  # noqa: BLE001
            errs[r] = e

    ts = [threading.Thread(target=rank, args=(r,)) for r in (0, 1)]
    for t in ts:
        t.start()
    ts[0].join(30)
    release.set()
    ts[1].join(30)
    assert isinstance(errs.get(0), TimeoutError), errs
    assert 1 not in errs
    assert keepalive[0] == 1
    assert groups[0].coll_timeout_s == 1.5
    # the timed-out group is closed: a later collective fails at once instead
    # of reading a stream a cut frame may have misaligned
    assert groups[0].broken == "timeout"
    with pytest.raises(ConnectionError):
        groups[0].barrier()
    for g in groups.values():
        g.close()
    # unbounded by default: a barrier behind a rank busy for any time passes
    if not os.environ.get("ANOMOD_HOSTGROUP_TIMEOUT_S"):
        assert dist.HostGroup(0, 1).coll_timeout_s is None


@pytest.mark.parametrize("refuse,uid_fails,expect", [
    ((False, False), False, "rccl"),
    ((True, True), False, "host"),    # RCCL refused everywhere (ranks sharing a device)
    ((False, True), False, "raise"),  # refused on one rank only: every rank raises
    ((False, False), True, "host"),   # rank 0 could not make the unique id
])
def test_attach_transport_agreement(tmp_path, monkeypatch, refuse, uid_fails, expect):
    """dist.attach (bench.py's transport choice): RCCL when every rank's
    communicator comes up, the host transport when RCCL refused on every rank,
    AnomodError on every rank when only some refused; a failed unique id on
    rank 0 reaches rank 1 as an empty broadcast, not a hang.  Fake contexts
    (no device): the agreement logic over a real two-rank HostGroup."""
    import threading

    from anomod import dist
    from anomod._lib import ERCCL, AnomodError

    def uid():
        if uid_fails:
            raise AnomodError(ERCCL, "ncclGetUniqueId failed")
        return b"u" * 128

    monkeypatch.setattr(dist.Context, "unique_id", staticmethod(uid))

    class FakeCtx:
        def __init__(self, refuse_init):
            self.refuse_init, self.comm, self.host = refuse_init, None, None

        def attach_comm(self, u, n, r):
            assert u == b"u" * 128
            if self.refuse_init:
                raise AnomodError(ERCCL, "ncclCommInitRank failed: invalid usage")
            self.comm = (n, r)

        def attach_host_comm(self, n, r, allreduce, allgather):
            self.host = (n, r)

    key, res, ctxs = f"attach{os.getpid()}", {}, {r: FakeCtx(refuse[r]) for r in (0, 1)}

    def rank(r):
        with dist.HostGroup(r, 2, key=key, rdzv_dir=str(tmp_path), timeout_s=30,
                            coll_timeout_s=30) as g:
            try:
                res[r] = dist.attach(ctxs[r], dist.RankInfo(r, 2, r), g)
            except AnomodError as e:
                res[r] = e

    ts = [threading.Thread(target=rank, args=(r,)) for r in (0, 1)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert set(res) == {0, 1}, res
    for r in (0, 1):
        if expect == "rccl":
            assert res[r] == "rccl" and ctxs[r].comm == (2, r) and ctxs[r].host is None
        elif expect == "host":
            assert res[r].startswith("host (RCCL refused") and ctxs[r].host == (2, r), res
        else:
            assert isinstance(res[r], AnomodError) and "up on 1 of 2" in str(res[r])
