"""Memory-bounded ("out-of-core") GEMM: host-resident operands streamed through the GPU.

Reference: ``src/zgemm_NN_gpu.jdf`` (C blocked into (tB P) x (tC Q) super-blocks,
K walked in chunks of tD tiles, LOCAL/GLOBAL barrier tasks capping the GPU
memory in use, C advised to GPU ``(n/Q) % ngpu``, :135-426) and its sizing /
dispatch in ``src/zgemm_wrapper.c:247-333,439-486`` (``dplasma_info`` keys
``DPLASMA:GEMM:GPU:{mem_ratio,c_ratio,look_ahead,b,c,d}``; chosen when the
active set would exceed GPU memory).

MI355X design: with 288 GB of HBM per GPU most problems are simply resident,
so this variant is for matrices that live in host memory (TiledMatrix on the
CPU) while the context drives a GPU.  C is processed in super-blocks of
b x c tiles held in a device tile arena; for each block the A / B tiles of a
K-chunk of d tiles are gathered into pinned staging buffers and uploaded on a
dedicated copy stream, double-buffered (look_ahead = 2) so chunk j+1 crosses
PCIe / the host link while chunk j runs in the batched MFMA GEMM kernel; the C
block goes back to host memory when its K loop ends.  Block sizes default to
the largest that fit ``mem_ratio`` of the free device memory.

Distributed (P x Q ranks, every operand host-resident and 2-D block-cyclic): the C super-blocks are
GLOBAL blocks of b x c tiles walked by every rank in the same order (the reference's LOCAL / GLOBAL
barrier structure); for each block and K-chunk, each rank receives the A tiles of its C rows and
the B tiles of its C columns that other ranks own -- only those: one planned all-to-all of exact
sizes (RCCL on device buffers, or gloo on host buffers), fed from the owners' host memory through
pinned staging -- uploads its own tiles, and runs one MFMA GEMM launch on its C tiles of the block.
"""
from __future__ import annotations

import math

import torch

from ..constants import STORAGE_TILE, dplasmaNoTrans
from ..ops import tile_ops as ops
from ..ops.batch import GemmBatch
from ..runtime.taskpool import Taskpool
from ..utils.flops import flops


def _a_tile(transA, m, k):
    return (m, k) if transA == dplasmaNoTrans else (k, m)


def _b_tile(transB, k, n):
    return (k, n) if transB == dplasmaNoTrans else (n, k)


def _sizes(ctx, A, B, C, kt, info):
    esz = C.data.element_size()
    tb = C.mb * C.nb * esz
    g = lambda k, d: info.get_int("DPLASMA:GEMM:GPU:" + k, d) if info is not None else d  # noqa: E731
    ratio = float(info.get_float("DPLASMA:GEMM:GPU:mem_ratio", 0.9)) if info is not None else 0.9
    la = max(1, g("look_ahead", 2))
    d = g("d", min(kt, 8))
    b, c = g("b", 0), g("c", 0)
    if not (b and c):
        free = torch.cuda.mem_get_info(ctx.device)[0]
        budget = max(ratio * free, 64 * tb)
        # b*c C tiles + la * d * (b + c) operand tiles <= budget / tb, with b == c
        x = budget / tb
        s = max(1, int((-la * d * 2 + math.sqrt((la * d * 2) ** 2 + 4 * x)) / 2))
        b, c = min(C.mt, s), min(C.nt, s)
    return max(1, b), max(1, c), max(1, d), la


class _GemmOOC(Taskpool):
    def __init__(self, ctx, transA, transB, alpha, A, B, beta, C, info):
        super().__init__("gemm_gpu", ctx)
        self.args = (transA, transB, alpha, A, B, beta, C)
        K = A.n if transA == dplasmaNoTrans else A.m
        self.kt = (K + (A.nb if transA == dplasmaNoTrans else A.mb) - 1) // (A.nb if transA == dplasmaNoTrans else A.mb)
        self.flops = flops(C.prec, "gemm", C.m, C.n, K)
        self.b, self.c, self.d, self.la = _sizes(ctx, A, B, C, self.kt, info)
        self.finish_build()

    def run(self, ctx=None):
        import time
        self._t_run = time.perf_counter()
        ctx = self.ctx
        transA, transB, alpha, A, B, beta, C = self.args
        dev = ctx.device
        dt = C.dtype
        ts = C.mb * C.nb
        b, c, d, la = self.b, self.c, self.d, self.la
        kext = (lambda k: A.tile_cols(k)) if transA == dplasmaNoTrans else (lambda k: A.tile_rows(k))
        comp = torch.cuda.current_stream(dev)
        copy = ctx.streams.get("aux") or torch.cuda.Stream(device=dev)
        nA, nB = b * d, d * c
        # device arenas: C block + look_ahead (A chunk, B chunk) buffers; pinned staging per buffer
        dC = torch.empty(b * c * ts, dtype=dt, device=dev)
        dA = [torch.empty(nA * ts, dtype=dt, device=dev) for _ in range(la)]
        dB = [torch.empty(nB * ts, dtype=dt, device=dev) for _ in range(la)]
        hA = [torch.empty(nA * ts, dtype=dt).pin_memory() for _ in range(la)]
        hB = [torch.empty(nB * ts, dtype=dt).pin_memory() for _ in range(la)]
        hC = torch.empty(b * c * ts, dtype=dt).pin_memory()
        ready = [torch.cuda.Event() for _ in range(la)]   # upload j done
        free = [None] * la                                # compute on buffer done

        def host_tile(M, i, j):
            return M.data[M.offset(i, j):M.offset(i, j) + ts] if M.storage == STORAGE_TILE else None

        def stage(M, tiles, host, slot_of):
            for (i, j), s in zip(tiles, slot_of):
                h = host_tile(M, i, j)
                dst = host[s * ts:(s + 1) * ts]
                if h is not None:
                    dst.copy_(h)
                else:  # LAPACK storage: pack the strided tile
                    t = M.tile(i, j)
                    torch.as_strided(dst, t.shape, (1, M.mb)).copy_(t)

        for m0 in range(0, C.mt, b):
            for n0 in range(0, C.nt, c):
                ms = list(range(m0, min(C.mt, m0 + b)))
                ns = list(range(n0, min(C.nt, n0 + c)))
                cslot = {(m, n): i * len(ns) + j for i, m in enumerate(ms) for j, n in enumerate(ns)}
                # C block in
                stage(C, list(cslot), hC, list(cslot.values()))
                with torch.cuda.stream(copy):
                    dC.copy_(hC, non_blocking=True)
                    evc = torch.cuda.Event()
                    evc.record(copy)
                comp.wait_event(evc)
                chunks = list(range(0, self.kt, d))
                for j, k0 in enumerate(chunks):
                    ks = list(range(k0, min(self.kt, k0 + d)))
                    buf = j % la
                    if free[buf] is not None:
                        free[buf].synchronize()          # host staging of this buffer is reusable
                    at = {(m, k): i * len(ks) + q for i, m in enumerate(ms) for q, k in enumerate(ks)}
                    bt = {(k, n): q * len(ns) + i for q, k in enumerate(ks) for i, n in enumerate(ns)}
                    stage(A, [_a_tile(transA, m, k) for (m, k) in at], hA[buf], list(at.values()))
                    stage(B, [_b_tile(transB, k, n) for (k, n) in bt], hB[buf], list(bt.values()))
                    with torch.cuda.stream(copy):
                        dA[buf].copy_(hA[buf], non_blocking=True)
                        dB[buf].copy_(hB[buf], non_blocking=True)
                        ready[buf].record(copy)
                    comp.wait_event(ready[buf])
                    gb = GemmBatch()
                    for (m, n), s in cslot.items():
                        kp = [(at[(m, k)] * ts, bt[(k, n)] * ts, kext(k)) for k in ks]
                        gb.add(s * ts, C.tile_rows(m), C.tile_cols(n), kp)
                    with torch.cuda.stream(comp):
                        ops.gemm(transA, transB, alpha, dA[buf], A.mb, dB[buf], B.mb, beta if j == 0 else 1.0,
                                 dC, C.mb, gb)
                    ev = torch.cuda.Event()
                    ev.record(comp)
                    free[buf] = ev
                # C block out
                ev = torch.cuda.Event()
                ev.record(comp)
                copy.wait_event(ev)
                with torch.cuda.stream(copy):
                    hC.copy_(dC, non_blocking=True)
                    evo = torch.cuda.Event()
                    evo.record(copy)
                evo.synchronize()
                for (m, n), s in cslot.items():
                    h = host_tile(C, m, n)
                    if h is not None:
                        h.copy_(hC[s * ts:(s + 1) * ts])
                    else:
                        t = C.tile(m, n)
                        t.copy_(torch.as_strided(hC[s * ts:(s + 1) * ts], t.shape, (1, C.mb)))
                comp.wait_stream(copy)

    def complete(self, ctx=None):
        torch.cuda.current_stream(self.ctx.device).synchronize()
        self._result = 0
        return 0


class _GemmOOCDist(Taskpool):
    """Host-resident, block-cyclic operands on P x Q ranks (see module docstring)."""

    def __init__(self, ctx, transA, transB, alpha, A, B, beta, C, info, sizes=None):
        super().__init__("gemm_gpu", ctx)
        self.args = (transA, transB, alpha, A, B, beta, C)
        K = A.n if transA == dplasmaNoTrans else A.m
        self.kt = -(-K // A.nb)
        self.flops = flops(C.prec, "gemm", C.m, C.n, K)
        if sizes is None:
            b, c, d, _ = _sizes(ctx, A, B, C, self.kt, info) if ctx.is_gpu else (4, 4, 2, 1)
            # the sizes bound MY share of a global block: scale by the grid
            g = C.grid
            b, c = b * g.P, c * g.Q
            if info is not None:   # explicit DPLASMA:GEMM:GPU:{b,c,d} are global block sizes
                b = info.get_int("DPLASMA:GEMM:GPU:b", b)
                c = info.get_int("DPLASMA:GEMM:GPU:c", c)
            sizes = (b, c, d)
        self.b, self.c, self.d = (max(1, x) for x in sizes)
        self.bytes_recv = 0     # elements received from other ranks (all blocks, all chunks)
        self.finish_build()

    def _exchange(self, needs, mats, ts):
        """needs[r]: ordered (mid, i, j) tiles rank r needs that it does not own -> my receive slab
        (device), in my need order grouped by source; owners pack from host memory."""
        import numpy as np
        import torch.distributed as dist
        ctx = self.ctx
        me, world = ctx.rank, ctx.world
        dev = ctx.device
        dt = mats[0].dtype
        owner = lambda key: mats[key[0]].rank_of(key[1], key[2])  # noqa: E731
        mine = needs[me]
        by_src = [[key for key in mine if owner(key) == s] for s in range(world)]
        order = [key for s in range(world) for key in by_src[s]]
        sends = [[key for key in needs[d] if owner(key) == me] for d in range(world)]
        nsend = sum(len(x) for x in sends)
        sbuf = torch.empty(max(1, nsend) * ts, dtype=dt, pin_memory=ctx.is_gpu)
        pos = 0
        for d in range(world):
            for (mid, i, j) in sends[d]:
                _pack(mats[mid], i, j, sbuf[pos * ts:(pos + 1) * ts])
                pos += 1
        rcount = [len(x) * ts for x in by_src]
        scount = [len(x) * ts for x in sends]
        nb_ = dist.get_backend() == "nccl"
        if ctx.is_gpu and nb_:
            dsend = sbuf.to(dev, non_blocking=True)
            rbuf = torch.empty(max(1, len(order)) * ts, dtype=dt, device=dev)
            dist.all_to_all_single(rbuf[: len(order) * ts], dsend[: nsend * ts], rcount, scount)
        else:
            rbuf = torch.empty(max(1, len(order)) * ts, dtype=dt)
            dist.all_to_all_single(rbuf[: len(order) * ts], sbuf[: nsend * ts], rcount, scount)
            rbuf = rbuf.to(dev)
        self.bytes_recv += len(order) * ts
        return {key: n * ts for n, key in enumerate(order)}, rbuf

    def run(self, ctx=None):
        import time
        self._t_run = time.perf_counter()
        ctx = self.ctx
        transA, transB, alpha, A, B, beta, C = self.args
        dev = ctx.device
        ts = C.mb * C.nb
        kext = (lambda k: A.tile_cols(k)) if transA == dplasmaNoTrans else (lambda k: A.tile_rows(k))
        g = C.grid
        mats = [A, B]
        world = ctx.world
        if beta != 1.0:
            for (m, n) in C.local_tiles():
                C.tile(m, n).mul_(beta)
        for m0 in range(0, C.mt, self.b):
            for n0 in range(0, C.nt, self.c):
                rows = list(range(m0, min(C.mt, m0 + self.b)))
                cols = list(range(n0, min(C.nt, n0 + self.c)))
                mytiles = [(m, n) for m in rows for n in cols if C.is_local(m, n)]
                cslot = {t: i * ts for i, t in enumerate(mytiles)}
                dC = torch.empty(max(1, len(mytiles)) * ts, dtype=C.dtype, device=dev)
                for (m, n), o in cslot.items():
                    _unpack_to(C, m, n, dC[o:o + ts])
                for j, k0 in enumerate(range(0, self.kt, self.d)):
                    ks = list(range(k0, min(self.kt, k0 + self.d)))
                    needs = {}
                    for r in range(world):
                        pr, pc = r // g.Q, r % g.Q
                        rr = [m for m in rows if g.prow(m + C.it0) == pr]
                        cc = [n for n in cols if g.pcol(n + C.jt0) == pc]
                        lst = []
                        for m in rr:
                            for k in ks:
                                i_, j_ = _a_tile(transA, m, k)
                                if A.rank_of(i_, j_) != r:
                                    lst.append((0, i_, j_))
                        for n in cc:
                            for k in ks:
                                i_, j_ = _b_tile(transB, k, n)
                                if B.rank_of(i_, j_) != r:
                                    lst.append((1, i_, j_))
                        needs[r] = lst
                    roff, rbuf = self._exchange(needs, mats, ts)
                    # my own operand tiles of the chunk
                    own = []
                    for m in sorted({m for (m, _) in mytiles}):
                        own += [(0,) + _a_tile(transA, m, k) for k in ks]
                    for n in sorted({n for (_, n) in mytiles}):
                        own += [(1,) + _b_tile(transB, k, n) for k in ks]
                    own = [key for key in own if mats[key[0]].rank_of(key[1], key[2]) == ctx.rank]
                    lbuf = torch.empty(max(1, len(own)) * ts, dtype=C.dtype, device=dev)
                    loff = {}
                    for n_, key in enumerate(own):
                        _unpack_to(mats[key[0]], key[1], key[2], lbuf[n_ * ts:(n_ + 1) * ts])
                        loff[key] = n_ * ts
                    # one launch per (A source, B source) pair
                    groups = {}
                    for (m, n), o in cslot.items():
                        for k in ks:
                            ka, kb = (0,) + _a_tile(transA, m, k), (1,) + _b_tile(transB, k, n)
                            sa = ("l", loff[ka]) if ka in loff else ("r", roff[ka])
                            sb = ("l", loff[kb]) if kb in loff else ("r", roff[kb])
                            groups.setdefault((sa[0], sb[0]), {}).setdefault((m, n), []).append((sa[1], sb[1],
                                                                                               kext(k)))
                    for (ga, gb_), items in sorted(groups.items()):
                        gbt = GemmBatch()
                        for (m, n), kp in items.items():
                            gbt.add(cslot[(m, n)], C.tile_rows(m), C.tile_cols(n), kp)
                        gbt.finalize()
                        # beta was applied to the host C tiles when the run started
                        ops.gemm(transA, transB, alpha, lbuf if ga == "l" else rbuf, C.mb,
                                 lbuf if gb_ == "l" else rbuf, C.mb, 1.0, dC, C.mb, gbt)
                for (m, n), o in cslot.items():
                    _pack_back(C, m, n, dC[o:o + ts])
        if ctx.is_gpu:
            torch.cuda.current_stream(dev).synchronize()

    def complete(self, ctx=None):
        if self.ctx.is_gpu:
            torch.cuda.current_stream(self.ctx.device).synchronize()
        self._result = 0
        return 0


def _pack(M, i, j, dst):
    """Host tile (i, j) of M -> dst (mb x nb slot, ld = mb)."""
    t = M.tile(i, j)
    torch.as_strided(dst, t.shape, (1, M.mb)).copy_(t)


def _unpack_to(M, i, j, dst):
    """Host tile -> device slot (zero padding past a ragged edge)."""
    t = M.tile(i, j)
    if t.shape != (M.mb, M.nb):
        dst.zero_()
    torch.as_strided(dst, t.shape, (1, M.mb)).copy_(t, non_blocking=False)


def _pack_back(M, i, j, src):
    t = M.tile(i, j)
    t.copy_(torch.as_strided(src, t.shape, (1, M.mb)))


def gemm_gpu_New(ctx, transA, transB, alpha, A, B, beta, C, info=None, allow_cpu=False) -> Taskpool:
    """C = alpha op(A) op(B) + beta C with A, B, C in host memory, computed on ctx's GPU in
    memory-bounded blocks (dplasma_zgemm_New_ex's GPU variant); any P x Q grid.
    ``allow_cpu``: run the distributed block / exchange schedule on a CPU context (tests)."""
    if not ctx.is_gpu and not allow_cpu:
        raise ValueError("gemm_gpu needs a GPU context")
    if not (A.mb == A.nb == B.mb == B.nb == C.mb == C.nb):
        raise ValueError("gemm_gpu needs square tiles of one size")
    if ctx.world > 1 or not ctx.is_gpu:
        sizes = None
        inf = info or ctx.info
        if inf is not None and inf.get_int("DPLASMA:GEMM:GPU:b", 0):
            sizes = (inf.get_int("DPLASMA:GEMM:GPU:b", 1), inf.get_int("DPLASMA:GEMM:GPU:c", 1),
                     inf.get_int("DPLASMA:GEMM:GPU:d", 1))
        return _GemmOOCDist(ctx, transA, transB, alpha, A, B, beta, C, inf, sizes)
    return _GemmOOC(ctx, transA, transB, alpha, A, B, beta, C, info or ctx.info)


def gemm_gpu(ctx, transA, transB, alpha, A, B, beta, C, info=None):
    gemm_gpu_New(ctx, transA, transB, alpha, A, B, beta, C, info).execute(ctx)
    return 0
