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


def bcast(t: torch.Tensor, src_global: int, group) -> None:
    if group is None:
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
