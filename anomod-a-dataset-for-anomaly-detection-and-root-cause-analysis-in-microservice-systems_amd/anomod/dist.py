"""Multi-GPU plumbing: one process per GPU, traceId-hash sharding, RCCL.

Traces are self-contained — parent resolution never crosses a trace
(_build_span_records runs per trace, trace_collector.py:531) — so a span
set shards by ``trace_hash % world`` with no data exchange; the only
collective is the integer all-reduce (sum / min / max) of the edge table
that libanomod issues itself once a communicator is attached.  The
reference has no distributed backend at all.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Callable

from .device import Context
from .spans import SpanSet


@dataclass
class RankInfo:
    rank: int
    world: int
    local_rank: int


def rank_from_env() -> RankInfo:
    """RANK / WORLD_SIZE / LOCAL_RANK as set by torch.distributed.run."""
    return RankInfo(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
                    int(os.environ.get("LOCAL_RANK", "0")))


def shard_spans(spans: SpanSet, info: RankInfo) -> SpanSet:
    return spans if info.world == 1 else spans.shard(info.world, info.rank)


def torch_exchange(uid: bytes | None) -> bytes:
    """Broadcast rank 0's RCCL unique id over an initialised torch.distributed
    group (any backend; the host-side rendezvous only)."""
    import torch.distributed as tdist

    obj = [uid]
    tdist.broadcast_object_list(obj, src=0)
    return obj[0]


def attach_rccl(ctx: Context, info: RankInfo,
                exchange: Callable[[bytes | None], bytes] = torch_exchange) -> None:
    """Create the RCCL communicator of this rank (no-op for world == 1)."""
    if info.world <= 1:
        return
    uid = Context.unique_id() if info.rank == 0 else None
    uid = exchange(uid)
    ctx.attach_comm(uid, info.world, info.rank)


def attach_gloo(ctx: Context, info: RankInfo) -> None:
    """Host transport over an initialised torch.distributed group (gloo):
    the libanomod collectives (status agreement, edge-table merge, sharded
    PageRank exchange) go through host memory instead of RCCL — for ranks
    that share one device, where RCCL refuses to run.  No-op for world == 1."""
    if info.world <= 1:
        return
    import numpy as np
    import torch
    import torch.distributed as tdist

    from . import _lib as L

    ops = {L.OP_SUM: tdist.ReduceOp.SUM, L.OP_MIN: tdist.ReduceOp.MIN,
           L.OP_MAX: tdist.ReduceOp.MAX}

    def allreduce(a: np.ndarray, dtype: int, op: int) -> None:
        if dtype == L.DTYPE_U64:
            if op != L.OP_SUM:
                raise ValueError("u64 min/max is not used by libanomod")
            t = torch.from_numpy(a.view(np.int64))  # two's complement: same bits mod 2^64
            tdist.all_reduce(t, ops[op])
        elif dtype == L.DTYPE_U32:  # widened: the u32 range is not a signed 32-bit one
            t = torch.from_numpy(a.astype(np.int64))
            tdist.all_reduce(t, ops[op])
            a[:] = t.numpy().astype(np.uint32)
        else:
            tdist.all_reduce(torch.from_numpy(a), ops[op])

    def allgather(a: np.ndarray, block: int) -> None:
        mine = torch.from_numpy(a[info.rank * block:(info.rank + 1) * block].copy())
        parts = [torch.empty(block, dtype=torch.uint8) for _ in range(info.world)]
        tdist.all_gather(parts, mine)
        for r, t in enumerate(parts):
            a[r * block:(r + 1) * block] = t.numpy()

    ctx.attach_host_comm(info.world, info.rank, allreduce, allgather)

