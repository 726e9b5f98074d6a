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


def _insert_potrf(tp, uplo, A, info):
    """The tile Cholesky as DTD tasks, with the reference's flushes (testing_zpotrf_dtd_untied.c)."""
    for _ in _potrf_steps(tp, uplo, A, info):
        pass


def _potrf_steps(tp, uplo, A, info):
    """Generator form of _insert_potrf: yields after every inserted task (the untied inserter stops
    and resumes between any two insertions)."""
    bases = [k * A.mb for k in range(A.mt)]
    ct = dplasmaConjTrans if A.dtype.is_complex else dplasmaTrans
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
    total = A.mt
    # priorities of the reference driver (tests/testing_zpotrf_dtd.c:134-186): cubic in the distance
    # to the end, the panel first
    for k in range(A.mt):
        tp.insert_task(potrf, (T(A, k, k), InOut | Aff), k, priority=(total - k) ** 3)
        yield
        for m in range(k + 1, A.mt):
            pr = (total - m) ** 3 + 3 * (2 * total - k - m - 1) * (m - k)
            if uplo == dplasmaLower:
                tp.insert_task(trsm, (T(A, k, k), In), (T(A, m, k), InOut | Aff), priority=pr)
            else:
                tp.insert_task(trsm, (T(A, k, k), In), (T(A, k, m), InOut | Aff), priority=pr)
            yield
        tp.data_flush(T(A, k, k))
        for m in range(k + 1, A.mt):
            pr = (total - m) ** 3 + 3 * (m - k)
            if uplo == dplasmaLower:
                tp.insert_task(herk, (T(A, m, k), In), (T(A, m, k), In), (T(A, m, m), InOut | Aff), priority=pr)
                yield
                for n in range(k + 1, m):
                    tp.insert_task(gemm, (T(A, m, k), In), (T(A, n, k), In), (T(A, m, n), InOut | Aff),
                                   priority=(total - m) ** 3 + 3 * (2 * total - m - n - 3) * (m - n) + 6 * (m - k))
                    yield
            else:
                tp.insert_task(herk, (T(A, k, m), In), (T(A, k, m), In), (T(A, m, m), InOut | Aff), priority=pr)
                yield
                for n in range(k + 1, m):
                    tp.insert_task(gemm, (T(A, k, n), In), (T(A, k, m), In), (T(A, n, m), InOut | Aff),
                                   priority=(total - m) ** 3 + 3 * (2 * total - m - n - 3) * (m - n) + 6 * (m - k))
                    yield
            tp.data_flush(T(A, m, k) if uplo == dplasmaLower else T(A, k, m))
    tp.flops = flops(A.prec, "potrf", A.m)
    tp.data_flush_all(A)


def _info_reducer(ctx, info):
    def _done():
        v = info.clone()
        if ctx.world > 1:
            import torch.distributed as dist
            dist.all_reduce(v, op=dist.ReduceOp.MAX)
        return int(v.item())
    return _done


def potrf_dtd_New(ctx, uplo, A):
    """Tile Cholesky through DTD insert_task (deferred: a compiled taskpool; result() = info)."""
    if A.mb != A.nb:
        raise ValueError("square tiles required")
    info = torch.zeros(1, dtype=torch.int32, device=A.device)
    tp = dtd.taskpool_new(ctx, "potrf_dtd", window=0)
    _insert_potrf(tp, uplo, A, info)
    ctp = tp.compile()
    ctp.on_complete(_info_reducer(ctx, info))
    return ctp


def potrf_dtd(ctx, uplo, A, window=None):
    """Blocking DTD Cholesky: windows of inserted tasks run while insertion continues."""
    if A.mb != A.nb:
        raise ValueError("square tiles required")
    info = torch.zeros(1, dtype=torch.int32, device=A.device)
    tp = dtd.taskpool_new(ctx, "potrf_dtd", window=window)
    tp.on_complete(_info_reducer(ctx, info))
    _insert_potrf(tp, uplo, A, info)
    r = tp.wait()
    potrf_dtd.last = tp
    return r


def untied_inserter(tp, steps, margin: int = 1000):
    """Body of the reference's untied inserter task (testing_zpotrf_dtd_untied.c:140-145): insert from
    the ``steps`` generator; once the window is nearly full, return AGAIN so the runtime launches what
    was inserted and calls the body again (the generator resumes where it stopped)."""
    lim = max(1, int(min(tp.window, 1 << 30)) - margin) if tp.window != float("inf") else None

    def body():
        for _ in steps:
            if lim is not None and tp.pending >= lim:
                return dtd.AGAIN
        return None
    return body


def potrf_dtd_untied(ctx, uplo, A, window=None):
    """The reference's untied variant (tests/testing_zpotrf_dtd_untied.c): ONE task without data is
    inserted; it runs on every rank and its body inserts the whole Cholesky into the taskpool it runs
    in, returning AGAIN whenever the window is nearly full."""
    info = torch.zeros(1, dtype=torch.int32, device=A.device)
    tp = dtd.taskpool_new(ctx, "potrf_dtd_untied", window=window)
    tp.on_complete(_info_reducer(ctx, info))
    margin = min(1000, max(1, int(min(tp.window, 1 << 30)) // 4))
    tp.insert_task(tp.task_class("insert_task_lower" if uplo == dplasmaLower else "insert_task_upper",
                                 untied_inserter(tp, _potrf_steps(tp, uplo, A, info), margin)))
    r = tp.wait()
    potrf_dtd_untied.last = tp
    return r


# ----------------------------------------------------------------------------- GEMM
def gemm_dtd(ctx, transA, transB, alpha, A, B, beta, C, window=None):
    """C = alpha op(A) op(B) + beta C through DTD insert_task (tests/testing_zgemm_dtd.c: one GEMM task
    per (m, n, k), the C tile's owner computes; k runs in order on each C tile)."""
    Ka = A.nt if transA == dplasmaNoTrans else A.mt
    tp = dtd.taskpool_new(ctx, "gemm_dtd", window=window)
    bodies = {}

    def body_for(beta_k):
        b = bodies.get(beta_k)
        if b is None:
            b = bodies[beta_k] = tp.task_class(f"gemm_b{beta_k}", _gemm_body(transA, transB, alpha, beta_k, 0))
        return b
    T = dtd.tile_of
    In, InOut, Aff = dtd.INPUT, dtd.INOUT, dtd.AFFINITY
    for m in range(C.mt):
        for n in range(C.nt):
            for k in range(Ka):
                ta = T(A, m, k) if transA == dplasmaNoTrans else T(A, k, m)
                tb = T(B, k, n) if transB == dplasmaNoTrans else T(B, n, k)
                tp.insert_task(body_for(beta if k == 0 else 1.0), (ta, In), (tb, In), (T(C, m, n), InOut | Aff))
    tp.flops = flops(C.prec, "gemm", C.m, C.n, A.n if transA == dplasmaNoTrans else A.m)
    tp.data_flush_all(C)
    tp.wait()
    gemm_dtd.last = tp
    return 0


def _blocking_New(name, ctx, fn, flops_):
    """A taskpool whose run inserts and executes a windowed DTD algorithm (insertion inside the timed
    region, concurrent with execution -- the reference's testing_z*_dtd drivers)."""
    from ..runtime.taskpool import Taskpool
    tp = Taskpool(name, ctx)
    tp.flops = flops_
    box = {}
    tp.task(name, "update", lambda: box.__setitem__("r", fn()))
    tp.on_complete(lambda: box.get("r"))
    return tp.finish_build()


def potrf_dtd_untied_New(ctx, uplo, A, window=None):
    return _blocking_New("potrf_dtd_untied", ctx, lambda: potrf_dtd_untied(ctx, uplo, A, window),
                         flops(A.prec, "potrf", A.m))


def gemm_dtd_New(ctx, transA, transB, alpha, A, B, beta, C, window=None):
    K = A.n if transA == dplasmaNoTrans else A.m
    return _blocking_New("gemm_dtd", ctx, lambda: gemm_dtd(ctx, transA, transB, alpha, A, B, beta, C, window),
                         flops(C.prec, "gemm", C.m, C.n, K))
