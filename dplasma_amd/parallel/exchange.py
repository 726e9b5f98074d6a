"""Planned many-to-many tile exchange (one all-to-all per exchange).

Every rank computes, from the (replicated) distribution metadata alone, the
same global plan: which tiles each rank needs and who owns them.  Executing
the plan packs the tiles a rank owns into a send slab (one batched copy
kernel), runs ONE ``all_to_all_single`` (RCCL over xGMI: direct point-to-point
transfers on every link at once; gloo on CPU), and leaves every needed tile in
a contiguous receive slab whose per-tile offsets are known at plan time, so
the consuming GEMM launch can address it directly.

This is the transport behind SUMMA GEMM, transposed additions, and the
redistribution used by the ScaLAPACK shims -- the role of PaRSEC's implicit
remote-dependency transfers and of ``parsec_redistribute``.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import torch
import torch.distributed as dist

from . import comm

from ..constants import dplasmaNoTrans
from ..ops import tile_ops as ops
from ..ops.batch import TileBatch

TileKey = Tuple[int, int, int]  # (matrix id, m, n)


class ExchangePlan:
    def __init__(self, ctx, mats: Sequence, needs: Dict[int, List[TileKey]], dtype, device):
        """mats: list of TiledMatrix indexed by matrix id; needs[r]: ordered tile keys rank r needs.

        Receive layout: the tiles of every REMOTE source in rank order (the all-to-all output), then my
        own tiles, which one batched copy moves straight from the matrix into their slots -- they never
        pass through the send slab or the collective (each local tile crosses HBM once)."""
        self.ctx = ctx
        self.mats = mats
        me = ctx.rank
        world = ctx.world
        mb = max(M.mb for M in mats)
        nb = max(M.nb for M in mats)
        self.nbe = nbe = mb * nb
        self.ld = mb
        mine = needs.get(me, [])
        # loopback rehearsal (parallel.comm.loopback): my own tiles go through the all-to-all as well
        self.loop = loop = bool(getattr(ctx, "loopback", False))
        by_src: List[List[TileKey]] = [[] for _ in range(world)]
        for key in mine:
            mid, m, n = key
            by_src[mats[mid].rank_of(m, n)].append(key)
        self.recv_counts = [len(x) if (s != me or loop) else 0 for s, x in enumerate(by_src)]
        self.slot: Dict[TileKey, int] = {}
        pos = 0
        order = list(range(world)) if loop else [x for x in range(world) if x != me] + [me]
        for s in order:
            for key in by_src[s]:
                self.slot[key] = pos * nbe
                pos += 1
        self.nrecv = pos
        self.nremote = pos if loop else pos - len(by_src[me])
        # my own tiles: matrix -> receive slot, one batch per source matrix
        self.local: Dict[int, TileBatch] = {}
        for (mid, m, n) in ([] if loop else by_src[me]):
            M = mats[mid]
            self.local.setdefault(mid, TileBatch()).add(M.offset(m, n), M.tile_rows(m), M.tile_cols(n),
                                                        b_off=self.slot[(mid, m, n)])
        for tb in self.local.values():
            tb.finalize()
        # send layout: by destination rank (never myself), in the destination's need order
        send_lists: List[List[TileKey]] = []
        for d in range(world):
            lst = [] if (d == me and not loop) else \
                [key for key in needs.get(d, []) if mats[key[0]].rank_of(key[1], key[2]) == me]
            send_lists.append(lst)
        self.send_counts = [len(x) for x in send_lists]
        self.nsend = sum(self.send_counts)
        self.pack: Dict[int, TileBatch] = {}
        p = 0
        for d in range(world):
            for (mid, m, n) in send_lists[d]:
                M = mats[mid]
                tb = self.pack.setdefault(mid, TileBatch())
                tb.add(M.offset(m, n), M.tile_rows(m), M.tile_cols(n), b_off=p * nbe)
                p += 1
        for tb in self.pack.values():
            tb.finalize()
        self.dtype, self.device = dtype, device

    def new_recv_buffer(self) -> torch.Tensor:
        return torch.empty(max(self.nrecv, 1) * self.nbe, dtype=self.dtype, device=self.device)

    def new_send_buffer(self) -> torch.Tensor:
        return torch.empty(max(self.nsend, 1) * self.nbe, dtype=self.dtype, device=self.device)

    def offset(self, mid: int, m: int, n: int) -> int:
        return self.slot[(mid, m, n)]

    def run(self, recv: torch.Tensor, sendbuf: torch.Tensor = None):
        """Pack + all-to-all into ``recv`` (on the current stream).  ``sendbuf``: a slab of at least
        ``nsend`` tiles the caller re-uses across runs (plans issued on one stream may share one)."""
        nbe = self.nbe
        for mid, tb in self.local.items():
            M = self.mats[mid]
            ops.geadd(0, dplasmaNoTrans, 1.0, M.data, M.ld, 0.0, recv, self.ld, tb, copy=True)
        if self.ctx.world == 1 and not self.loop:
            return
        if sendbuf is None or sendbuf.numel() < self.nsend * nbe:
            sendbuf = self.new_send_buffer()
        for mid, tb in self.pack.items():
            M = self.mats[mid]
            ops.geadd(0, dplasmaNoTrans, 1.0, M.data, M.ld, 0.0, sendbuf, self.ld, tb, copy=True)
        out_splits = [c * nbe for c in self.recv_counts]
        in_splits = [c * nbe for c in self.send_counts]
        comm._rec_coll("alltoall", None, None)
        w = dist.all_to_all_single(recv[: self.nremote * nbe], sendbuf[: self.nsend * nbe], out_splits,
                                   in_splits, async_op=True)
        w.wait()
