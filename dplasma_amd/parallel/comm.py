"""Tile transport between ranks (one process per GPU).

Backed by ``torch.distributed``: RCCL (backend "nccl") over xGMI on GPU,
gloo on CPU.  Collectives are issued from inside a taskpool task, i.e. with
the task's stream current: the collective waits for that stream's prior
work, and ``work.wait()`` makes the stream (not the host) wait for the
transfer, so communication overlaps the other streams' compute.

Patterns used by the algorithms (SURVEY.md §2.10 collective inventory):
* ``bcast``      -- panel diagonal tile to the owner column, panel piece
                    along a process row (direct fan-out; RCCL picks the
                    algorithm per message size);
* ``allgather``  -- panel pieces across a process column (in place);
* ``allreduce``  -- info / norm reductions.

Loopback rehearsal (``DPLASMA_LOOPBACK=1`` on a world-1 process group): the algorithms plan
their exchanges as if the rank's own tiles lived on another rank -- every tile edge that would
cross ranks on a real grid (and, for tile DAGs / tile programs, every operand edge) becomes a
send to and a receive from the rank itself.  On RCCL those are real ``ncclSend`` / ``ncclRecv``
pairs in one group (NCCL supports self-sends; only torch's Python front end refuses them,
``_check_not_self_rank``, which :func:`self_p2p` lifts for the duration of the call), so every
RCCL branch of the transport (grouped p2p batches, the urgent / bulk communicators, the
dataflow ``Transport`` of tile DAGs, all-to-all exchanges) executes on a one-GPU box with
results that must equal the exchange-free path.  gloo cannot connect a rank to itself: there
the self pairs are completed by a local copy (the CPU tests check the planning).
"""
from __future__ import annotations

import contextlib
import os
from typing import Optional

import torch
import torch.distributed as dist


def _nbytes(t: torch.Tensor) -> int:
    return t.numel() * t.element_size()


def loopback() -> bool:
    """True when the loopback rehearsal is on: DPLASMA_LOOPBACK=1 and a world-1 process group."""
    return (os.environ.get("DPLASMA_LOOPBACK", "0") == "1" and dist.is_available() and dist.is_initialized()
            and dist.get_world_size() == 1)


@contextlib.contextmanager
def self_p2p():
    """Let torch.distributed post sends / receives whose peer is this rank (loopback only)."""
    if not loopback():
        yield
        return
    import torch.distributed.distributed_c10d as c10d
    orig = c10d._check_not_self_rank
    c10d._check_not_self_rank = lambda *a, **k: None
    try:
        yield
    finally:
        c10d._check_not_self_rank = orig


def _split_self(sends, recvs):
    """gloo loopback: complete the self pairs (in order) with local copies; returns the rest."""
    me = dist.get_rank() if dist.is_initialized() else 0
    ss = [t for t, p in sends if p == me]
    rs = [t for t, p in recvs if p == me]
    if len(ss) != len(rs):
        raise RuntimeError(f"loopback: {len(ss)} self-sends but {len(rs)} self-receives in one batch")
    for a, b in zip(ss, rs):
        b.copy_(a.view(-1)[: b.numel()].view_as(b))
    return [(t, p) for t, p in sends if p != me], [(t, p) for t, p in recvs if p != me]


def bcast(t: torch.Tensor, src_global: int, group, world: bool = False) -> None:
    """Broadcast from global rank src_global over ``group`` (None: nothing to do -- unless ``world``,
    then over every rank)."""
    if _BACKEND is not None and hasattr(_BACKEND, "sync"):
        return _BACKEND.sync("bcast", _nbytes(t), group)
    if group is None and not world:
        return
    if world and not (dist.is_initialized() and dist.get_world_size() > 1):
        return
    w = dist.broadcast(t, src=src_global, group=group, async_op=True)
    w.wait()


def _nccl() -> bool:
    return dist.get_backend() == "nccl"


def allgather_inplace(out: torch.Tensor, my_index: int, group) -> None:
    """out is [n_in_group, ...] contiguous; slot my_index already holds my contribution."""
    if _BACKEND is not None and hasattr(_BACKEND, "sync"):
        return _BACKEND.sync("allgather", _nbytes(out) - _nbytes(out[my_index]), group)
    if group is None:
        return
    inp = out[my_index]
    if out.device.type == "cuda" and _nccl():
        w = dist.all_gather_into_tensor(out.view(-1), inp.reshape(-1),
                                        group=group, async_op=True)
        w.wait()
    else:
        parts = list(out.unbind(0))
        mine = inp.clone()
        w = dist.all_gather(parts, mine, group=group, async_op=True)
        w.wait()


def allreduce(t: torch.Tensor, op=dist.ReduceOp.SUM, group=None) -> None:
    if _BACKEND is not None and hasattr(_BACKEND, "sync"):
        return _BACKEND.sync("allreduce", 2 * _nbytes(t), group)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    dist.all_reduce(t, op=op, group=group)


def p2p(sends=(), recvs=()) -> None:
    """Grouped point-to-point transfer: sends / recvs are lists of (tensor, global peer rank).

    RCCL: one grouped send/recv call (every pair on its own xGMI link); the current stream waits
    for the transfer.  gloo: CUDA tensors are staged through host memory (gloo moves host buffers)."""
    sends, recvs = list(sends), list(recvs)
    if not sends and not recvs:
        return
    if _BACKEND is not None and hasattr(_BACKEND, "sync"):
        per = {}
        for t_, p_ in sends + recvs:
            per[p_] = per.get(p_, 0) + _nbytes(t_)
        return _BACKEND.sync("p2p", max(per.values()), None)
    if _nccl():
        ops = [dist.P2POp(dist.isend, t, p) for t, p in sends] + [dist.P2POp(dist.irecv, t, p) for t, p in recvs]
        with self_p2p():
            for w in dist.batch_isend_irecv(ops) or ():
                w.wait()
        return
    if loopback():
        sends, recvs = _split_self(sends, recvs)
    host_r = [(t, t.cpu() if t.device.type != "cpu" else t) for t, _ in recvs]
    works = [dist.isend(t.cpu() if t.device.type != "cpu" else t, p) for t, p in sends]
    works += [dist.irecv(h, p) for (_, h), (_, p) in zip(host_r, recvs)]
    for w in works:
        w.wait()
    for t, h in host_r:
        if h is not t:
            t.copy_(h)


class Pending:
    """An exchange in flight (``start_p2p``), completed by ``finish`` on the consumer's side.
    Device transfers (RCCL) are waited for per consumer stream; host ones (gloo) once."""
    __slots__ = ("works", "host_recvs", "keep", "device", "streams", "done", "meta")

    def __init__(self, works, host_recvs=(), keep=(), device=False, meta=None):
        self.works, self.host_recvs, self.keep = list(works), list(host_recvs), keep
        self.device, self.streams, self.done, self.meta = device, set(), False, meta


_BACKEND = None   # replaces the torch.distributed transport (tools/replay_potrf.py: modelled xGMI timing)


def set_backend(b) -> None:
    """Install a transport backend with ``start_p2p(sends, recvs, group, hint)`` / ``finish(p)`` and
    optionally ``sync(kind, critical_bytes, group)`` for the blocking collectives (None: torch.distributed)."""
    global _BACKEND
    _BACKEND = b


def start_p2p(sends=(), recvs=(), group=None, hint=None) -> Optional[Pending]:
    """Issue a grouped point-to-point exchange and return at once.

    sends / recvs: lists of (tensor, global peer rank); ``group``: the process group whose
    communicator carries it (each group has its own RCCL stream, so exchanges on different groups
    proceed concurrently -- over different xGMI links when their peers differ).  RCCL: the transfer
    waits for the current stream's prior work and runs on the group's stream; ``finish`` (issued
    later, under the consumer's stream) makes that stream -- not the host -- wait.  gloo: CUDA
    tensors are staged through host memory; ``finish`` waits on the host and unstages.
    ``hint`` describes the producer's work for a modelling backend; the real transports ignore it."""
    sends, recvs = list(sends), list(recvs)
    if not sends and not recvs:
        return None
    if _BACKEND is not None:
        return _BACKEND.start_p2p(sends, recvs, group, hint)
    if _nccl() and any(t.device.type == "cuda" for t, _ in sends + recvs):
        ops = [dist.P2POp(dist.isend, t, p, group=group) for t, p in sends]
        ops += [dist.P2POp(dist.irecv, t, p, group=group) for t, p in recvs]
        with self_p2p():
            return Pending(dist.batch_isend_irecv(ops) or (), device=True)
    if loopback():
        sends, recvs = _split_self(sends, recvs)
    host_s = [(t.cpu() if t.device.type != "cpu" else t, p) for t, p in sends]
    host_r = [(t, t.cpu() if t.device.type != "cpu" else t, p) for t, p in recvs]
    works = [dist.isend(h, p, group=group) for h, p in host_s]
    works += [dist.irecv(h, p, group=group) for _, h, p in host_r]
    return Pending(works, [(t, h) for t, h, _ in host_r if h is not t], keep=host_s)


def finish(p: Optional[Pending]) -> None:
    """Complete an exchange from ``start_p2p`` for the caller: RCCL -- the current stream waits for
    the transfer (once per stream); gloo -- the host waits and unstages (once).  None: no-op."""
    if p is None or p.done:
        return
    if p.device:
        sid = torch.cuda.current_stream().cuda_stream
        if sid in p.streams:
            return
        p.streams.add(sid)
        if _BACKEND is not None:
            _BACKEND.finish(p)
        else:
            for w in p.works:
                w.wait()
        return
    if _BACKEND is not None:
        _BACKEND.finish(p)
    else:
        for w in p.works:
            w.wait()
        for t, h in p.host_recvs:
            t.copy_(h)
    p.done = True


def exchange_add(t: torch.Tensor, peer: int, tmp: torch.Tensor) -> None:
    """t += (peer's t): symmetric pairwise sum through one send/recv pair (tmp: same size as t)."""
    p2p([(t, peer)], [(tmp[: t.numel()], peer)])
    t.add_(tmp[: t.numel()])


_TRI_IDX = {}


def _tri_index(n: int, ld: int, lower: bool, device) -> torch.Tensor:
    """Element offsets (column-major, leading dimension ld) of the lower / upper triangle of an n x n
    block, diagonal included -- n (n + 1) / 2 entries."""
    key = (n, ld, lower, str(device))
    t = _TRI_IDX.get(key)
    if t is None:
        r = torch.arange(n).view(-1, 1)
        c = torch.arange(n).view(1, -1)
        mask = (r >= c) if lower else (r <= c)
        off = (r + c * ld).expand(n, n)
        t = _TRI_IDX[key] = off.t()[mask.t()].contiguous().to(device)   # column by column
    return t


def bcast_tri(dst: torch.Tensor, dst_off: int, src: Optional[torch.Tensor], src_off: int, n: int, ld_src: int,
              ld_dst: int, lower: bool, root: int, group, pack: Optional[torch.Tensor] = None) -> None:
    """Broadcast only the lower / upper triangle of an n x n block (the reference's LOWER_TILE /
    UPPER_TILE arena shapes: half the bytes of the full tile).  The root reads its block from
    ``src[src_off]`` (leading dimension ld_src); every rank (root included) gets the triangle in
    ``dst[dst_off]`` (ld_dst); the rest of the destination block is not written."""
    if _BACKEND is not None and hasattr(_BACKEND, "sync"):
        return _BACKEND.sync("bcast", n * (n + 1) // 2 * dst.element_size(), group)
    if group is None:
        return
    nt = n * (n + 1) // 2
    buf = pack[:nt] if pack is not None else torch.empty(nt, dtype=dst.dtype, device=dst.device)
    if src is not None:
        buf.copy_(src.view(-1)[src_off + _tri_index(n, ld_src, lower, src.device)])
    bcast(buf, root, group)
    dst.view(-1)[dst_off + _tri_index(n, ld_dst, lower, dst.device)] = buf
