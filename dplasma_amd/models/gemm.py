"""Distributed GEMM: C = alpha op(A) op(B) + beta C.

Reference: ``src/zgemm_wrapper.c`` dispatching to the default
(``zgemm_{NN,NT,TN,TT}.jdf``), SUMMA (``zgemm_*_summa.jdf``: RING_A/RING_B
rings along process rows/columns with look-ahead CTLs, :91-207) and the
out-of-GPU-memory variant (``zgemm_NN_gpu.jdf``).

MI355X design:
* Single rank: the whole product is ONE launch of the batched MFMA GEMM
  engine -- every local C tile is an item whose k-loop runs over all k tiles
  inside the kernel (no per-k launches, C read and written exactly once).
* P x Q ranks (SUMMA): K is cut into chunks of ``kc`` tile columns; for each
  chunk one planned all-to-all (``parallel.exchange``) delivers the A tiles of
  my C rows and the B tiles of my C columns (any transpose, any distribution),
  then one GEMM launch accumulates the chunk.  Chunks are double-buffered: the
  exchange of chunk s+1 (panel stream) overlaps the GEMM of chunk s (update
  stream); ``DPLASMA:GEMM:look_ahead`` chunks may be in flight (default from
  utils.aux.gemm_lookahead).  With 288 GB of HBM per GPU the default chunk is
  large (fewer, larger collectives), see ``DPLASMA:GEMM:kc``.
"""
from __future__ import annotations

import torch

from ..constants import dplasmaNoTrans
from ..ops import tile_ops as ops
from ..ops.batch import MASK_LOWER, MASK_UPPER, GemmBatch
from ..parallel.exchange import ExchangePlan
from ..runtime import Taskpool
from ..utils.flops import flops


def _check(transA, transB, A, B, C):
    am, ak = (A.m, A.n) if transA == dplasmaNoTrans else (A.n, A.m)
    bk, bn = (B.m, B.n) if transB == dplasmaNoTrans else (B.n, B.m)
    if am != C.m or bn != C.n or ak != bk:
        raise ValueError(f"gemm: size mismatch op(A)={am}x{ak} op(B)={bk}x{bn} C={C.m}x{C.n}")
    return ak


def _a_tile(transA, m, k):
    return (m, k) if transA == dplasmaNoTrans else (k, m)


def _b_tile(transB, k, n):
    return (k, n) if transB == dplasmaNoTrans else (n, k)


def gemm_New(ctx, transA, transB, alpha, A, B, beta, C, c_mask=None, kc=None, name="gemm") -> Taskpool:
    """c_mask(m, n) -> MASK_* restricts the update of C tile (m,n) to a triangle (used by herk/syrk).

    Host-resident operands with a GPU context dispatch to the memory-bounded
    streaming variant (models/gemm_ooc.py), like dplasma_zgemm_New_ex picks the
    GPU variant when the active set exceeds GPU memory (src/zgemm_wrapper.c:455-486)."""
    K = _check(transA, transB, A, B, C)
    if (ctx.is_gpu and c_mask is None and C.device.type == "cpu"
            and A.device.type == "cpu" and B.device.type == "cpu"):
        from .gemm_ooc import gemm_gpu_New
        return gemm_gpu_New(ctx, transA, transB, alpha, A, B, beta, C)
    tp = Taskpool(name, ctx)
    tp.flops = flops(C.prec, "gemm", C.m, C.n, K)
    kt = (K + A.nb - 1) // A.nb if transA == dplasmaNoTrans else (K + A.mb - 1) // A.mb
    # tile size along k (op(A) columns)
    def kext(k):
        return A.tile_cols(k) if transA == dplasmaNoTrans else A.tile_rows(k)
    ctiles = [(m, n) for (m, n) in C.local_tiles() if c_mask is None or c_mask(m, n) is not None]
    # distributed: a rank without C tiles may still own A/B tiles others need, so it
    # must join every exchange -- only kt == 0 (identical on all ranks) skips them
    single = ctx.world == 1 and not getattr(ctx, "loopback", False)
    if kt == 0 or (not ctiles and single):
        if beta != 1.0 and ctiles:
            from .aux import lascal_New
            return lascal_New(ctx, 123, beta, C)
        return tp.finish_build()
    if single:
        gb = GemmBatch()
        for (m, n) in ctiles:
            kp = [(A.offset(*_a_tile(transA, m, k)), B.offset(*_b_tile(transB, k, n)), kext(k)) for k in range(kt)]
            gb.add(C.offset(m, n), C.tile_rows(m), C.tile_cols(n), kp, c_mask(m, n) if c_mask else 0)
        gb.finalize()
        tp.task("GEMM", "update", lambda: ops.gemm(transA, transB, alpha, A.data, A.ld, B.data, B.ld, beta, C.data,
                                                     C.ld, gb))
        return tp.finish_build()
    # ---------------- SUMMA over k chunks
    if kc is None:
        kc = ctx.info.get_int("DPLASMA:GEMM:kc", 0) or max(1, min(kt, 8))
    nchunks = (kt + kc - 1) // kc
    # look-ahead: chunks whose exchange may run ahead of the GEMM consuming the oldest one
    # (reference DPLASMA:GEMM:GPU:look_ahead, src/zgemm_wrapper.c:289-296; the SUMMA look-ahead
    # CTLs of zgemm_NN_summa.jdf); one receive buffer per chunk in flight
    from ..utils.aux import gemm_lookahead
    la = ctx.info.get_int("DPLASMA:GEMM:look_ahead", 0) or ctx.info.get_int("DPLASMA:GEMM:GPU:look_ahead", 0) \
        or gemm_lookahead(ctx, C)
    if la <= 0:
        raise ValueError("DPLASMA:GEMM:look_ahead must be 1 or more")
    nbuf = min(nchunks, la + 1)
    mats = [A, B]
    bufs = []
    prev_gemm = {}
    plans = []
    for s in range(nchunks):
        ks = list(range(s * kc, min(kt, (s + 1) * kc)))
        needs = {}
        for r in range(ctx.world):
            pr, pc = r // C.Q, r % C.Q
            rows = [m for m in range(C.mt) if C.grid.prow(m + C.it0) == pr]
            cols = [n for n in range(C.nt) if C.grid.pcol(n + C.jt0) == pc]
            lst = []
            for m in rows:
                for k in ks:
                    lst.append((0,) + _a_tile(transA, m, k))
            for n in cols:
                for k in ks:
                    lst.append((1,) + _b_tile(transB, k, n))
            needs[r] = lst
        plan = ExchangePlan(ctx, mats, needs, C.dtype, C.device)
        if len(bufs) < nbuf:
            bufs.append(plan.new_recv_buffer())
        buf = bufs[s % nbuf]
        if buf.numel() < max(plan.nrecv, 1) * plan.nbe:
            buf = plan.new_recv_buffer()
            bufs[s % nbuf] = buf
        gb = GemmBatch()
        for (m, n) in ctiles:
            kp = [(plan.offset(0, *_a_tile(transA, m, k)), plan.offset(1, *_b_tile(transB, k, n)), kext(k))
                  for k in ks]
            gb.add(C.offset(m, n), C.tile_rows(m), C.tile_cols(n), kp, c_mask(m, n) if c_mask else 0)
        gb.finalize()
        plans.append(plan)
        # one send slab for every chunk: the exchanges are issued in order on the panel stream
        t_ex = tp.task(f"EXCH({s})", "panel", lambda plan=plan, buf=buf: plan.run(buf, tp._sendbuf),
                       [prev_gemm.get(s - nbuf)], prio=2)
        b_eff = beta if s == 0 else 1.0
        prev_gemm[s] = tp.task(
            f"GEMM({s})", "update",
            lambda gb=gb, buf=buf, b_eff=b_eff, plan=plan: ops.gemm(transA, transB, alpha, buf, plan.ld, buf, plan.ld, b_eff,
                                                          C.data, C.ld, gb), [t_ex], prio=1)
    tp._buffers = bufs
    tp._sendbuf = torch.empty(max([p.nsend for p in plans] + [1]) * plans[0].nbe, dtype=C.dtype, device=C.device)
    return tp.finish_build()


def gemm(ctx, transA, transB, alpha, A, B, beta, C, **kw):
    return gemm_New(ctx, transA, transB, alpha, A, B, beta, C, **kw).execute(ctx)
