"""Memory-capped Cholesky: a host-resident matrix factored through a bounded GPU tile arena.

Reference: the PaRSEC GPU device memory manager the reference relies on -- a fixed pool of device
blocks, tiles staged in on demand and written back / evicted LRU when the pool is full -- and its
low-memory test (tests/Testings.cmake:147: ``potrf ... 1gpu_lowmem -N 3200 -t 320 -- --mca
device_cuda_memory_number_of_blocks 21``).

MI355X design: with 288 GB of HBM per GPU the normal path keeps the whole matrix resident; this
variant is for a TiledMatrix that lives in host memory while the context drives a GPU (or for a
capped arena requested with ``DPLASMA:GPU:number_of_blocks`` / the ``nblocks`` argument).
:class:`TileCache` owns ``nblocks`` device tile slots: ``get(tile, write)`` returns a resident
slot, uploading the tile if needed and evicting the least recently used unpinned slot (dirty
slots are written back first); ``flush()`` writes every dirty slot home.  The factorisation walks
the right-looking tile algorithm (POTRF(k), TRSM(m,k), SYRK/GEMM(m,n,k)) and pins the <= 3 tiles a
task touches, so any arena of >= 3 slots completes; each task is one tile-kernel launch of the
device engine (potrf_tile / trsm / gemm batches of one item).  Copies run on the compute stream
(pinned host staging), so the arena is reused without cross-stream hazards.
"""
from __future__ import annotations

from collections import OrderedDict

import torch

from ..constants import dplasmaConjTrans, dplasmaLeft, dplasmaLower, dplasmaNoTrans, dplasmaNonUnit, dplasmaRight
from ..ops import tile_ops as ops
from ..ops.batch import MASK_LOWER, MASK_UPPER, GemmBatch, TileBatch
from ..runtime import Taskpool
from ..utils.flops import flops


class TileCache:
    """LRU arena of ``nblocks`` mb x nb tile slots on ``device`` backed by host tiles of ``A``."""

    def __init__(self, A, nblocks: int, device):
        if nblocks < 3:
            raise ValueError("memory-capped mode needs at least 3 tile slots")
        self.A = A
        self.device = torch.device(device)
        self.nbe = A.mb * A.nb
        self.ld = A.mb
        self.arena = torch.zeros(nblocks * self.nbe, dtype=A.dtype, device=self.device)
        self.free = list(range(nblocks))
        self.slot = OrderedDict()      # tile -> slot (LRU order: oldest first)
        self.dirty = set()
        self.pinned = set()
        self.loads = self.evictions = self.writebacks = 0
        pin = self.device.type == "cuda"
        self.stage = torch.empty(self.nbe, dtype=A.dtype, pin_memory=pin)

    def view(self, s: int, t):
        r, c = self.A.tile_rows(t[0]), self.A.tile_cols(t[1])
        return torch.as_strided(self.arena, (r, c), (1, self.ld), s * self.nbe)

    def off(self, t) -> int:
        return self.slot[t] * self.nbe

    def _writeback(self, t, s):
        self.A.tile(*t).copy_(self.view(s, t))
        self.writebacks += 1

    def get(self, t, write: bool = False) -> int:
        """Element offset in the arena of resident tile t (pinned until release())."""
        if t in self.slot:
            self.slot.move_to_end(t)
        else:
            if not self.free:
                victim = next((v for v in self.slot if v not in self.pinned), None)
                if victim is None:
                    raise RuntimeError("tile arena exhausted by pinned tiles")
                vs = self.slot.pop(victim)
                if victim in self.dirty:
                    self._writeback(victim, vs)
                    self.dirty.discard(victim)
                self.evictions += 1
                self.free.append(vs)
            s = self.free.pop()
            self.slot[t] = s
            self.view(s, t).copy_(self.A.tile(*t), non_blocking=False)
            self.loads += 1
        if write:
            self.dirty.add(t)
        self.pinned.add(t)
        return self.off(t)

    def release(self):
        self.pinned.clear()

    def flush(self):
        for t in list(self.dirty):
            self._writeback(t, self.slot[t])
        self.dirty.clear()


def potrf_ooc_New(ctx, uplo: int, A, nblocks: int = 0) -> Taskpool:
    """Cholesky of the host-resident (or any) A through a device arena of ``nblocks`` tiles."""
    if A.grid.P * A.grid.Q != 1:
        raise ValueError("memory-capped potrf: single-process descriptors only")
    lower = uplo == dplasmaLower
    nt = A.nt
    if nblocks <= 0:
        nblocks = ctx.info.get_int("DPLASMA:GPU:number_of_blocks", 0)
    if nblocks <= 0:
        free = torch.cuda.mem_get_info(ctx.device)[0] if ctx.is_gpu else 1 << 34
        nblocks = max(3, min(nt * (nt + 1) // 2, int(0.8 * free) // (A.mb * A.nb * A.data.element_size())))
    tp = Taskpool("potrf_ooc", ctx)
    tp.flops = flops(A.prec, "potrf", A.n)
    info = torch.zeros(1, dtype=torch.int32, device=ctx.device)
    tp.info = info
    tA, tB = (dplasmaNoTrans, dplasmaConjTrans) if lower else (dplasmaConjTrans, dplasmaNoTrans)

    def tc(i, k):  # panel coordinate -> tile
        return (i, k) if lower else (k, i)

    def body():
        cache = TileCache(A, nblocks, ctx.device)
        tp.cache = cache
        ar, ld = cache.arena, cache.ld
        for k in range(nt):
            kb = A.tile_rows(k)
            o = cache.get(tc(k, k), write=True)
            ops.potrf_tile(uplo, ar, o, kb, ld, info, k * A.mb)
            cache.release()
            for i in range(k + 1, nt):
                od = cache.get(tc(k, k))
                ob = cache.get(tc(i, k), write=True)
                tb = TileBatch()
                if lower:
                    tb.add(od, A.tile_rows(i), kb, b_off=ob)
                else:
                    tb.add(od, kb, A.tile_cols(i), b_off=ob)
                ops.trsm(dplasmaRight if lower else dplasmaLeft, uplo, dplasmaConjTrans, dplasmaNonUnit, 1.0,
                         ar, ld, ar, ld, tb.finalize())
                cache.release()
            for n in range(k + 1, nt):
                for m in range(n, nt):
                    on = cache.get(tc(n, k))
                    om = cache.get(tc(m, k))
                    cc = tc(m, n)
                    oc = cache.get(cc, write=True)
                    gb = GemmBatch()
                    # lower: C(m,n) -= L(m,k) L(n,k)^H ; upper: C(n,m) -= U(k,n)^H U(k,m)
                    gb.add(oc, A.tile_rows(cc[0]), A.tile_cols(cc[1]), [(om, on, kb) if lower else (on, om, kb)],
                           (MASK_LOWER if lower else MASK_UPPER) if m == n else 0)
                    ops.gemm(tA, tB, -1.0, ar, ld, ar, ld, 1.0, ar, ld, gb.finalize())
                    cache.release()
        cache.flush()

    tp.task("POTRF_OOC", "update", body, [])

    def _done():
        return int(info.item())
    tp.on_complete(_done)
    return tp.finish_build()


def potrf_ooc(ctx, uplo: int, A, nblocks: int = 0) -> int:
    return potrf_ooc_New(ctx, uplo, A, nblocks).execute(ctx)
