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
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist


def bcast(t: torch.Tensor, src_global: int, group, world: bool = False) -> None:
    """Broadcast from global rank src_global over ``group`` (None: nothing to do -- unless ``world``,
    then over every rank)."""
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
    if _nccl():
        ops = [dist.P2POp(dist.isend, t, p) for t, p in sends] + [dist.P2POp(dist.irecv, t, p) for t, p in recvs]
        for w in dist.batch_isend_irecv(ops) or ():
            w.wait()
        return
    host_r = [(t, t.cpu() if t.device.type != "cpu" else t) for t, _ in recvs]
    works = [dist.isend(t.cpu() if t.device.type != "cpu" else t, p) for t, p in sends]
    works += [dist.irecv(h, p) for (_, h), (_, p) in zip(host_r, recvs)]
    for w in works:
        w.wait()
    for t, h in host_r:
        if h is not t:
            t.copy_(h)


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
    if group is None:
        return
    nt = n * (n + 1) // 2
    buf = pack[:nt] if pack is not None else torch.empty(nt, dtype=dst.dtype, device=dst.device)
    if src is not None:
        buf.copy_(src.view(-1)[src_off + _tri_index(n, ld_src, lower, src.device)])
    bcast(buf, root, group)
    dst.view(-1)[dst_off + _tri_index(n, ld_dst, lower, dst.device)] = buf
