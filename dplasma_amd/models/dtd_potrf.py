"""Cholesky written against the DTD insert-task interface.

Reference: ``src/dtd_wrappers/zpotrf.c:151-171`` and ``tests/testing_zpotrf_dtd.c``
(POTRF / TRSM / HERK / GEMM tasks inserted in loop order with
PARSEC_INPUT/INOUT|AFFINITY tiles).  Bodies call the same HIP tile kernels as
the optimized POTRF (one-item batches), so this path doubles as the runtime's
end-to-end DTD test; the batched stream program in ``models/potrf.py`` remains
the fast path.
"""
from __future__ import annotations

import torch

from ..constants import (dplasmaConjTrans, dplasmaLeft, dplasmaLower, dplasmaNoTrans, dplasmaNonUnit, dplasmaRight,
                         dplasmaTrans, dplasmaUpper)
from ..ops import tile_ops as ops
from ..ops.batch import MASK_LOWER, MASK_UPPER, GemmBatch, TileBatch
from ..runtime import dtd
from ..utils.flops import flops


def tile_args(v: torch.Tensor):
    """(flat base, element offset, ld) of a tile view, as the tile kernels expect."""
    n = v.untyped_storage().nbytes() // v.element_size()
    return v.as_strided((n,), (1,), 0), v.storage_offset(), v.stride(1)


def _potrf_body(uplo, info, base):
    def body(a, k):
        b, off, ld = tile_args(a)
        ops.potrf_tile(uplo, b, off, a.shape[0], ld, info, base[k])
    return body


def _trsm_body(side, uplo, trans):
    def body(t, x):
        tb, toff, tld = tile_args(t)
        xb, xoff, xld = tile_args(x)
        batch = TileBatch().add(toff, x.shape[0], x.shape[1], b_off=xoff).finalize()
        ops.trsm(side, uplo, trans, dplasmaNonUnit, 1.0, tb, tld, xb, xld, batch)
    return body


def _gemm_body(ta, tb_, alpha, beta, mask):
    def body(a, b, c):
        ab, aoff, ald = tile_args(a)
        bb, boff, bld = tile_args(b)
        cb, coff, cld = tile_args(c)
        k = a.shape[1] if ta == dplasmaNoTrans else a.shape[0]
        gb = GemmBatch().add(coff, c.shape[0], c.shape[1], [(aoff, boff, k)], mask).finalize()
        ops.gemm(ta, tb_, alpha, ab, ald, bb, bld, beta, cb, cld, gb)
    return body


def potrf_dtd_New(ctx, uplo, A):
    """Tile Cholesky through DTD insert_task (returns a compiled taskpool; result() = info)."""
    if A.mb != A.nb:
        raise ValueError("square tiles required")
    info = torch.zeros(1, dtype=torch.int32, device=A.device)
    bases = [k * A.mb for k in range(A.mt)]
    ct = dplasmaConjTrans if A.dtype.is_complex else dplasmaTrans
    tp = dtd.taskpool_new(ctx, "potrf_dtd")
    potrf = tp.task_class("potrf", _potrf_body(uplo, info, bases))
    if uplo == dplasmaLower:
        trsm = tp.task_class("trsm", _trsm_body(dplasmaRight, dplasmaLower, ct))
        herk = tp.task_class("herk", _gemm_body(dplasmaNoTrans, ct, -1.0, 1.0, MASK_LOWER))
        gemm = tp.task_class("gemm", _gemm_body(dplasmaNoTrans, ct, -1.0, 1.0, 0))
    else:
        trsm = tp.task_class("trsm", _trsm_body(dplasmaLeft, dplasmaUpper, ct))
        herk = tp.task_class("herk", _gemm_body(ct, dplasmaNoTrans, -1.0, 1.0, MASK_UPPER))
        gemm = tp.task_class("gemm", _gemm_body(ct, dplasmaNoTrans, -1.0, 1.0, 0))
    T = dtd.tile_of
    In, InOut, Aff = dtd.INPUT, dtd.INOUT, dtd.AFFINITY
    for k in range(A.mt):
        tp.insert_task(potrf, (T(A, k, k), InOut | Aff), k)
        for m in range(k + 1, A.mt):
            if uplo == dplasmaLower:
                tp.insert_task(trsm, (T(A, k, k), In), (T(A, m, k), InOut | Aff))
            else:
                tp.insert_task(trsm, (T(A, k, k), In), (T(A, k, m), InOut | Aff))
        for m in range(k + 1, A.mt):
            if uplo == dplasmaLower:
                tp.insert_task(herk, (T(A, m, k), In), (T(A, m, k), In), (T(A, m, m), InOut | Aff))
                for n in range(k + 1, m):
                    tp.insert_task(gemm, (T(A, m, k), In), (T(A, n, k), In), (T(A, m, n), InOut | Aff))
            else:
                tp.insert_task(herk, (T(A, k, m), In), (T(A, k, m), In), (T(A, m, m), InOut | Aff))
                for n in range(k + 1, m):
                    tp.insert_task(gemm, (T(A, k, n), In), (T(A, k, m), In), (T(A, n, m), InOut | Aff))
    tp.flops = flops(A.prec, "potrf", A.m)
    ctp = tp.compile()

    def _done():
        v = info.clone()
        if ctx.world > 1:
            import torch.distributed as dist
            dist.all_reduce(v, op=dist.ReduceOp.MAX)
        return int(v.item())
    ctp.on_complete(_done)
    return ctp


def potrf_dtd(ctx, uplo, A):
    return potrf_dtd_New(ctx, uplo, A).execute(ctx)
