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
