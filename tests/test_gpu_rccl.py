"""GPU: the RCCL merge of the edge table through libanomod's
own communicator.

* one rank: a 1-rank communicator runs the same ncclGroupStart / AllReduce
  (u64 sum, u32 min, u32 max) / GroupEnd sequence as N ranks;
* two ranks: two processes (one per GPU when the box has two, else both on
  GPU 0), the unique id through a stdlib TCP HostGroup (as bench.py does), traceId-hash
  shards, merged table == the oracle's unsharded table bit for bit.  RCCL
  refuses two ranks on one device ("invalid usage", measured on the 1-GPU
  box); that refusal is reported as a skip with RCCL's own message.
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


def test_one_rank_communicator_merge():
    sp = anomod.synth_generate_host(anomod.SynthSpec("SN", seed=5, p_orphan_ppm=3000), 20000)
    with anomod.Context(0) as c:
        c.attach_comm(anomod.Context.unique_id(), 1, 0)
        got = c.edge_aggregate(sp)
    assert_table_equal(got, native.edge_aggregate(sp, len(sp.services)))


_WORKER = textwrap.dedent("""
    import os, sys
    sys.path[:0] = [{pkg!r}, {root!r}]
    import numpy as np
    import anomod
    from anomod import dist
    info = dist.rank_from_env()
    grp = dist.HostGroup(info.rank, info.world)
    sp = anomod.synth_generate_host(anomod.SynthSpec("SN", seed=9, p_orphan_ppm=3000), 30000)
    part = dist.shard_spans(sp, info)
    with anomod.Context(info.rank % anomod.device_count()) as c:
        if {fallback!r}:
            tr = dist.attach(c, info, grp)
        else:
            dist.attach_rccl(c, info, grp)
            tr = "rccl"
        t = c.edge_aggregate(part)
    with open(os.path.join({out!r}, f"transport{{info.rank}}.txt"), "w") as f:
        f.write(tr)
    np.savez(os.path.join({out!r}, f"rank{{info.rank}}.npz"), count=t.count, errors=t.errors,
             sum_us=t.sum_us, min_us=t.min_us, max_us=t.max_us, hist=t.hist,
             p50_us=t.p50_us, p99_us=t.p99_us, n_part=part.n_spans)
    grp.barrier()
    grp.close()
""")


@pytest.mark.parametrize("fallback", [False, True])
def test_two_ranks_one_device(tmp_path, fallback):
    """fallback: bench.py's dist.attach — RCCL where it comes up, else (two
    ranks on the one GPU of this box, which RCCL refuses on both) the host
    transport, said in the returned string; the merged table is the oracle's
    either way."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    script = tmp_path / "worker.py"
    script.write_text(_WORKER.format(pkg=str(PKG_DIR), root=str(ROOT), out=str(tmp_path),
                                     fallback=fallback))
    procs = []
    for r in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                   WORLD_SIZE="2", LOCAL_RANK=str(r), NCCL_DEBUG="WARN")
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      start_new_session=True))
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=90)[0].decode(errors="replace"))
        except subprocess.TimeoutExpired:
            for q in procs:
                if q.poll() is None:
                    os.killpg(q.pid, 9)
            pytest.fail("two-rank RCCL run timed out")
    if any(p.returncode != 0 for p in procs):
        text = "\n".join(outs)
        if not fallback and ("uplicate GPU" in text or "invalid usage" in text):
            pytest.skip("RCCL refuses two ranks on one device: " + text[-300:])
        pytest.fail(text[-2000:])
    sp = anomod.synth_generate_host(anomod.SynthSpec("SN", seed=9, p_orphan_ppm=3000), 30000)
    ref = native.edge_aggregate(sp, len(sp.services))
    r0, r1 = (np.load(tmp_path / f"rank{r}.npz") for r in range(2))
    assert int(r0["n_part"]) + int(r1["n_part"]) == sp.n_spans
    assert 0 < int(r0["n_part"]) < sp.n_spans
    tr = [(tmp_path / f"transport{r}.txt").read_text() for r in range(2)]
    assert tr[0].split(" ")[0] == tr[1].split(" ")[0] in ("rccl", "host"), tr
    if fallback and anomod.device_count() == 1:
        assert tr[0].startswith("host (RCCL refused"), tr
    for r in (r0, r1):
        got = anomod.EdgeTable(services=sp.services, **{k: r[k] for k in (
            "count", "errors", "sum_us", "min_us", "max_us", "hist", "p50_us", "p99_us")})
        assert_table_equal(got, ref)
