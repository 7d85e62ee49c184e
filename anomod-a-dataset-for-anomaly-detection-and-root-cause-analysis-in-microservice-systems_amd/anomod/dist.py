"""Multi-GPU plumbing: one process per GPU, traceId-hash sharding, RCCL.

Traces are self-contained — parent resolution never crosses a trace
(_build_span_records runs per trace, trace_collector.py:531) — so a span
set shards by ``trace_hash % world`` with no data exchange; the only
collective is the integer all-reduce (sum / min / max) of the edge table
that libanomod issues itself once a communicator is attached.  The
reference has no distributed backend at all.

The host side needs no framework: ``HostGroup`` is a stdlib TCP group
(rank 0 serves, the other ranks connect) that carries the 128-B RCCL unique
id, the bench's barriers and scalar reductions, and — for ranks that share
one device, where RCCL refuses to run — libanomod's host collective
transport.  Rendezvous: rank 0 binds an ephemeral port and publishes it in a
file keyed by MASTER_PORT and the launcher's pid (every rank of one
``torch.distributed.run`` / test launch is a child of the same process), so
nothing collides with the launcher's own store on MASTER_PORT.
"""
from __future__ import annotations

import json
import os
import socket
import struct
import tempfile
import time
from dataclasses import dataclass
from pathlib import Path
from typing import Callable

import numpy as np

from ._lib import ERCCL, OP_MAX, OP_MIN, OP_SUM, AnomodError
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


# ---- stdlib TCP group ---------------------------------------------------------

_MAGIC = b"ANMD"


def _send(sock: socket.socket, data: bytes) -> None:
    sock.sendall(struct.pack("<Q", len(data)) + data)


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray(n)
    view = memoryview(buf)
    got = 0
    while got < n:
        k = sock.recv_into(view[got:], n - got)
        if k == 0:
            raise ConnectionError("peer closed the anomod host group")
        got += k
    return bytes(buf)


def _recv(sock: socket.socket) -> bytes:
    (n,) = struct.unpack("<Q", _recv_exact(sock, 8))
    return _recv_exact(sock, n)


def _reduce(parts: list[np.ndarray], op: int) -> np.ndarray:
    if op == OP_SUM:
        out = parts[0].copy()
        for p in parts[1:]:
            out += p  # unsigned integers wrap mod 2^bits, as the device sums do
        return out
    if op == OP_MIN:
        return np.minimum.reduce(parts)
    if op == OP_MAX:
        return np.maximum.reduce(parts)
    raise ValueError(f"unknown reduction op {op}")


def _link_options(sock: socket.socket, timeout_s: float | None) -> None:
    """A formed peer link: every recv bounded by timeout_s (None: unbounded),
    TCP keepalive on (probes after 30 s idle, every 10 s, 6 unanswered = dead
    link)."""
    sock.settimeout(timeout_s)
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_KEEPALIVE, 1)
    for name, v in (("TCP_KEEPIDLE", 30), ("TCP_KEEPINTVL", 10), ("TCP_KEEPCNT", 6)):
        if hasattr(socket, name):
            sock.setsockopt(socket.IPPROTO_TCP, getattr(socket, name), v)


class HostGroup:
    """A star-shaped TCP process group over the ranks of one node.

    Every collective gathers the ranks' payloads at rank 0, which combines
    them in rank order and sends the result back, so all ranks hold the same
    bytes.  Payloads here are tiny (an RCCL unique id, scalars) or the
    host-transport buffers of tests on one device."""

    def __init__(self, rank: int, world: int, key: str | None = None,
                 timeout_s: float | None = None, rdzv_dir: str | None = None,
                 coll_timeout_s: float | None = None):
        """timeout_s bounds the rendezvous (ANOMOD_RCCL_TIMEOUT_S, 300 s).
        Once the group is formed a collective waits for its peers without a
        bound by default, so a barrier behind a rank busy with local work for
        any time still passes; coll_timeout_s (or ANOMOD_HOSTGROUP_TIMEOUT_S)
        bounds that wait, after which it raises TimeoutError.  A rank that
        exits closes its socket, which every peer sees at once; a lost host
        stops answering TCP keepalive on every peer link (probes after 30 s,
        dead after ~90 s), which ends the wait with an error.  A collective
        that fails (timeout, closed or dead link) closes the group: a frame
        may have been cut, so later collectives raise ConnectionError instead
        of reading a misaligned stream."""
        if world < 1 or not 0 <= rank < world:
            raise ValueError(f"bad rank {rank} of world {world}")
        self.rank, self.world = rank, world
        self.timeout_s = float(timeout_s if timeout_s is not None
                               else os.environ.get("ANOMOD_RCCL_TIMEOUT_S", "300"))
        if coll_timeout_s is None:
            env = os.environ.get("ANOMOD_HOSTGROUP_TIMEOUT_S")
            coll_timeout_s = float(env) if env else None
        if coll_timeout_s is not None and not coll_timeout_s > 0:
            raise ValueError(f"collective timeout must be > 0 s, got {coll_timeout_s}")
        self.coll_timeout_s = None if coll_timeout_s is None else float(coll_timeout_s)
        self.broken: str | None = None  # why a failed collective closed the group
        self._peers: list[socket.socket] = []  # rank 0: ranks 1..world-1 in order
        self._sock: socket.socket | None = None  # other ranks: the link to rank 0
        self._file: Path | None = None
        if world == 1:
            return
        if key is None:
            key = f"{os.environ.get('MASTER_PORT', '0')}-{os.getppid()}"
        d = Path(rdzv_dir or os.environ.get("ANOMOD_RDZV_DIR") or tempfile.gettempdir())
        path = d / f"anomod-rdzv-{key}.json"
        host = os.environ.get("ANOMOD_RDZV_ADDR", "127.0.0.1")
        deadline = time.monotonic() + self.timeout_s
        if rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.bind((host, 0))
            srv.listen(world)
            tmp = path.with_suffix(f".tmp{os.getpid()}")
            tmp.write_text(json.dumps({"addr": host, "port": srv.getsockname()[1],
                                       "world": world, "pid": os.getpid()}))
            os.replace(tmp, path)
            self._file = path
            peers: dict[int, socket.socket] = {}
            try:
                while len(peers) < world - 1:
                    srv.settimeout(max(0.1, deadline - time.monotonic()))
                    try:
                        c, _ = srv.accept()
                    except socket.timeout:
                        raise TimeoutError(f"anomod host group: {len(peers) + 1} of {world} "
                                           f"ranks joined within {self.timeout_s:.0f} s") from None
                    # a stray or stale client that stalls, closes or sends
                    # garbage is dropped, not fatal to the rendezvous
                    c.settimeout(min(5.0, max(0.1, deadline - time.monotonic())))
                    try:
                        c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                        hello = _recv(c)
                        magic, r, w = hello[:4], *struct.unpack("<ii", hello[4:12])
                    except (OSError, ConnectionError, struct.error):
                        c.close()
                        continue
                    if magic != _MAGIC or w != world or not 0 < r < world or r in peers:
                        c.close()
                        continue
                    peers[r] = c
            except BaseException:
                for c in peers.values():
                    c.close()
                raise
            finally:
                srv.close()
            self._peers = [peers[r] for r in range(1, world)]
            for c in self._peers:
                _link_options(c, self.coll_timeout_s)
                _send(c, b"ok")
        else:
            while True:
                s = None
                try:
                    info = json.loads(path.read_text())
                    s = socket.create_connection((info["addr"], info["port"]), timeout=5.0)
                    s.settimeout(max(0.1, deadline - time.monotonic()))
                    s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    _send(s, _MAGIC + struct.pack("<ii", rank, world))
                    if _recv(s) == b"ok":
                        _link_options(s, self.coll_timeout_s)
                        self._sock, s = s, None
                        break
                except (OSError, ValueError, KeyError, ConnectionError, struct.error):
                    pass  # not published yet, or a stale file of an earlier run
                finally:
                    if s is not None:
                        s.close()
                if time.monotonic() > deadline:
                    raise TimeoutError(f"anomod host group: rank {rank} found no rank 0 at "
                                       f"{path} within {self.timeout_s:.0f} s")
                time.sleep(0.05)

    @classmethod
    def from_env(cls, **kw) -> "HostGroup":
        info = rank_from_env()
        return cls(info.rank, info.world, **kw)

    # -- primitives
    def _gather_bcast(self, payload: bytes, combine: Callable[[list[bytes]], bytes]) -> bytes:
        """Every rank's payload to rank 0, combine(payloads in rank order) back
        to every rank."""
        if self.world == 1:
            return combine([payload])
        if self.broken is not None:
            raise ConnectionError(f"anomod host group: closed after a failed collective "
                                  f"({self.broken})")
        try:
            if self.rank == 0:
                out = combine([payload] + [_recv(c) for c in self._peers])
                for c in self._peers:
                    _send(c, out)
                return out
            _send(self._sock, payload)
            return _recv(self._sock)
        except socket.timeout:
            self._fail("timeout")
            raise TimeoutError(f"anomod host group: rank {self.rank} of {self.world} waited "
                               f"{self.coll_timeout_s:.0f} s for a peer in a collective "
                               f"(ANOMOD_HOSTGROUP_TIMEOUT_S)") from None
        except (OSError, ConnectionError) as e:
            self._fail(type(e).__name__)
            raise

    def _fail(self, why: str) -> None:
        """A collective failed part-way: its frames may be cut, so the links
        are closed and the group refuses later collectives."""
        self.broken = why
        for c in self._peers:
            c.close()
        if self._sock is not None:
            self._sock.close()

    def broadcast(self, data: bytes | None, src: int = 0) -> bytes:
        """src's bytes on every rank."""
        mine = (b"\x01" + data) if self.rank == src else b"\x00"
        return self._gather_bcast(mine, lambda ps: next(p[1:] for p in ps if p[:1] == b"\x01"))

    def barrier(self) -> None:
        self._gather_bcast(b"", lambda ps: b"")

    def allreduce(self, a: np.ndarray, op: int = OP_SUM) -> None:
        """Reduce a numpy array in place over all ranks (same shape/dtype)."""
        dt, shape = a.dtype, a.shape

        def combine(ps):
            return _reduce([np.frombuffer(p, dtype=dt) for p in ps], op).tobytes()

        a[...] = np.frombuffer(self._gather_bcast(np.ascontiguousarray(a).tobytes(), combine),
                               dtype=dt).reshape(shape)

    def allgather(self, a: np.ndarray, block: int) -> None:
        """Every rank's ``block``-byte slice of the u8 array ``a`` (rank r's is
        a[r*block:(r+1)*block], set by rank r) on every rank."""
        mine = a[self.rank * block:(self.rank + 1) * block].tobytes()
        out = self._gather_bcast(mine, lambda ps: b"".join(ps))
        a[:block * self.world] = np.frombuffer(out, dtype=np.uint8)

    def allreduce_scalar(self, v: float, op: int = OP_SUM) -> float:
        t = np.array([v], dtype=np.float64)
        self.allreduce(t, op)
        return float(t[0])

    def close(self) -> None:
        for c in self._peers:
            c.close()
        if self._sock is not None:
            self._sock.close()
        self._peers, self._sock = [], None
        if self._file is not None:
            try:
                self._file.unlink()
            except OSError:
                pass
            self._file = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


# ---- libanomod communicators ------------------------------------------------------

def attach_rccl(ctx: Context, info: RankInfo,
                exchange: Callable[[bytes | None], bytes] | HostGroup | None = None) -> None:
    """Create the RCCL communicator of this rank (no-op for world == 1).
    Rank 0's 128-B unique id travels through ``exchange``: a HostGroup (its
    broadcast), any callable uid -> uid, or None = a HostGroup made from the
    environment for this call."""
    if info.world <= 1:
        return
    uid = Context.unique_id() if info.rank == 0 else None
    if isinstance(exchange, HostGroup):
        uid = exchange.broadcast(uid)
    elif exchange is not None:
        uid = exchange(uid)
    else:
        with HostGroup(info.rank, info.world) as g:
            uid = g.broadcast(uid)
    ctx.attach_comm(uid, info.world, info.rank)


def attach(ctx: Context, info: RankInfo, group: HostGroup, fallback: bool = True) -> str:
    """This rank's collective transport: RCCL when every rank's communicator
    comes up, else — when RCCL refused on every rank (ranks sharing one device,
    a node without peer access) and ``fallback`` — the host transport over
    ``group`` (attach_host).  Every rank reaches the same answer (one
    HostGroup sum of the successes), and a refusal on some ranks only raises
    AnomodError on all of them.  A failed unique id on rank 0 reaches the
    others as an empty broadcast instead of leaving them waiting.  Returns
    "rccl", "host (RCCL refused: ...)" or "none" (world == 1)."""
    if info.world <= 1:
        return "none"
    uid, err = None, ""
    if info.rank == 0:
        try:
            uid = Context.unique_id()
        except AnomodError as e:
            err = str(e)
    uid = group.broadcast(uid if uid is not None else b"")
    ok = 0.0
    if uid:
        try:
            ctx.attach_comm(uid, info.world, info.rank)
            ok = 1.0
        except AnomodError as e:
            err = str(e)
    else:
        err = err or "rank 0 could not make the RCCL unique id"
    n_ok = int(group.allreduce_scalar(ok, OP_SUM))
    if n_ok == info.world:
        return "rccl"
    if n_ok > 0 or not fallback:
        raise AnomodError(ERCCL, f"RCCL communicator up on {n_ok} of {info.world} "
                          f"ranks (this rank: {err or 'up'})")
    attach_host(ctx, group)
    return f"host (RCCL refused: {err[-200:]})"


def attach_host(ctx: Context, group: HostGroup) -> None:
    """Host collective transport over a HostGroup: the libanomod collectives
    (status agreement, edge-table merge, sharded PageRank exchange) go
    through host memory instead of RCCL — for ranks that share one device,
    where RCCL refuses to run.  No-op for world == 1."""
    if group.world <= 1:
        return
    ctx.attach_host_comm(group.world, group.rank, lambda a, _dtype, op: group.allreduce(a, op),
                         group.allgather)
