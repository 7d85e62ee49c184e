"""Multi-rank path on CPU (world_size 2, gloo): traceId-hash sharding plus the
integer sum/min/max merge the GPU path does with RCCL must reproduce the
unsharded edge table bit for bit.  The per-rank partial tables come from the
CPU oracle here (no GPU in this container); the sharding is the product's
(anomod.dist / SpanSet.shard)."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as tdist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank: int, world: int, port: int, out_dir: str):
    import sys

    from conftest import PKG_DIR, ROOT
    for p in (str(PKG_DIR), str(ROOT)):
        if p not in sys.path:
            sys.path.insert(0, p)
    import anomod
    from anomod import dist
    from oracle import native

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    info = dist.rank_from_env()
    assert (info.rank, info.world) == (rank, world)
    spans = anomod.synth_generate_host(anomod.SynthSpec("SN", seed=77, p_orphan_ppm=2000), 6000)
    part = dist.shard_spans(spans, info)
    tab = native.edge_aggregate(part, len(spans.services))
    for key, op in (("count", tdist.ReduceOp.SUM), ("errors", tdist.ReduceOp.SUM),
                    ("sum_us", tdist.ReduceOp.SUM), ("hist", tdist.ReduceOp.SUM),
                    ("min_us", tdist.ReduceOp.MIN), ("max_us", tdist.ReduceOp.MAX)):
        t = torch.from_numpy(tab[key].astype(np.int64))
        tdist.all_reduce(t, op=op)
        tab[key] = t.numpy()
    # an RCCL-style unique id handed to attach_rccl's exchange hook over gloo
    # (the product's default is dist.HostGroup: tests/test_dist_host.py)
    obj = [bytes(range(128)) if rank == 0 else None]
    tdist.broadcast_object_list(obj, src=0)
    assert obj[0] == bytes(range(128))
    if rank == 0:
        np.savez(os.path.join(out_dir, "merged.npz"), n_part=part.n_spans, **tab)
    tdist.barrier()
    tdist.destroy_process_group()


def test_two_rank_shard_merge_equals_whole(tmp_path):
    import anomod
    from oracle import native

    world, port = 2, _free_port()
    mp.start_processes(_worker, args=(world, port, str(tmp_path)), nprocs=world,
                       start_method="spawn")
    merged = np.load(tmp_path / "merged.npz")
    spans = anomod.synth_generate_host(anomod.SynthSpec("SN", seed=77, p_orphan_ppm=2000), 6000)
    whole = native.edge_aggregate(spans)
    for key in ("count", "errors", "sum_us", "hist", "max_us"):
        np.testing.assert_array_equal(merged[key].astype(np.uint64), whole[key], err_msg=key)
    mn = merged["min_us"].astype(np.int64)
    np.testing.assert_array_equal(mn.astype(np.uint32), whole["min_us"])
    assert 0 < int(merged["n_part"]) < spans.n_spans
