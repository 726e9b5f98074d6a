"""Tile QR and incremental-pivoting LU written against the DTD insert-task interface.

Reference: ``tests/testing_zgeqrf_dtd.c`` / ``testing_zgeqrf_dtd_untied.c`` (GEQRT / UNMQR / TSQRT /
TSMQR tasks inserted in loop order on A and the T tiles, the untied variant inserting from inside a
task) and ``tests/testing_zgetrf_incpiv_dtd.c`` (GETRF / GESSM / TSTRF / SSSSM on A, L and IPIV).

The task classes carry the batched tile kinds of the PTG-style tile DAGs (``ops/qr_ops.py``,
``ops/lu_incpiv_ops.py``: HIP launches on the GPU, the PyTorch transcription on the CPU): the ready
tasks of one class in a window level run as ONE launch, and the DTD factorizations store exactly what
the tile engines store -- V and T in the reference's per-tile TSQRT layout, L / IPIV in the
incremental-pivoting layout that ``trsmpl_incpiv`` consumes.
"""
from __future__ import annotations

import torch

from ..ops import lu_incpiv_ops, qr_ops
from ..runtime import dtd
from ..utils.flops import flops
from .dtd_potrf import _blocking_New, _info_reducer


# ----------------------------------------------------------------------------- QR
def _insert_geqrf(tp, A, T):
    """Flat-tree tile QR (zgeqrf.jdf task classes) as DTD tasks on A and T (ib x nb tiles)."""
    for _ in _geqrf_steps(tp, A, T):
        pass


def _geqrf_steps(tp, A, T):
    """Generator form of _insert_geqrf (yields after every inserted task)."""
    kd = qr_ops.kinds(A.dtype, T.mb, qr_ops.view_flags(A.dtype, False), qr_ops.view_flags(A.dtype, False))
    tc = {k: tp.task_class(k, kind=kd[k]) for k in ("geqrt", "unmqr_h", "tsqrt", "tsmqr_h")}
    Tl = dtd.tile_of
    In, InOut, Aff = dtd.INPUT, dtd.INOUT, dtd.AFFINITY
    for k in range(min(A.mt, A.nt)):
        ck, rk = A.tile_cols(k), A.tile_rows(k)
        tp.insert_task(tc["geqrt"], (Tl(A, k, k), InOut | Aff), (Tl(T, k, k), InOut), (rk, ck, 0))
        yield
        for n in range(k + 1, A.nt):
            # roles C, V, T
            tp.insert_task(tc["unmqr_h"], (Tl(A, k, n), InOut | Aff), (Tl(A, k, k), In), (Tl(T, k, k), In),
                           (rk, A.tile_cols(n), min(rk, ck)))
            yield
        for m in range(k + 1, A.mt):
            rm = A.tile_rows(m)
            # roles A1, A2, T -- executed where A2 (the killed tile) lives
            tp.insert_task(tc["tsqrt"], (Tl(A, k, k), InOut), (Tl(A, m, k), InOut | Aff), (Tl(T, m, k), InOut),
                           (rm, ck, 0))
            yield
            for n in range(k + 1, A.nt):
                # roles A1, A2, V, T
                tp.insert_task(tc["tsmqr_h"], (Tl(A, k, n), InOut), (Tl(A, m, n), InOut | Aff), (Tl(A, m, k), In),
                               (Tl(T, m, k), In), (rm, A.tile_cols(n), ck))
                yield
        tp.data_flush(Tl(A, k, k))
    T.full_T = {}   # per-tile T factors (the stacked-domain engine's kept factors do not describe T)
    T.qr_format = "tile"
    tp.data_flush_all(A)
    tp.data_flush_all(T)


def _check_qr(A, T):
    if A.mb != A.nb:
        raise ValueError("square tiles required")
    if T.nb != A.nb or T.mb > 64 or T.mt < A.mt or T.nt < A.nt:
        raise ValueError("T must have mt x nt tiles of ib x nb (ib <= 64)")


def geqrf_dtd(ctx, A, T, window=None):
    """Blocking DTD tile QR (tests/testing_zgeqrf_dtd.c): windows run while insertion continues."""
    _check_qr(A, T)
    tp = dtd.taskpool_new(ctx, "geqrf_dtd", window=window)
    tp.flops = flops(A.prec, "geqrf", A.m, A.n)
    _insert_geqrf(tp, A, T)
    tp.wait()
    geqrf_dtd.last = tp
    return 0


def geqrf_dtd_untied(ctx, A, T, window=None):
    """Untied variant (tests/testing_zgeqrf_dtd_untied.c): one inserted task without data runs on every
    rank and inserts the whole QR into the taskpool it runs in (AGAIN when the window is nearly full)."""
    from .dtd_potrf import untied_inserter
    _check_qr(A, T)
    tp = dtd.taskpool_new(ctx, "geqrf_dtd_untied", window=window)
    tp.flops = flops(A.prec, "geqrf", A.m, A.n)

    def steps():
        yield from _geqrf_steps(tp, A, T)
    margin = min(1000, max(1, int(min(tp.window, 1 << 30)) // 4))
    tp.insert_task(tp.task_class("insert_tasks", untied_inserter(tp, steps(), margin)))
    tp.wait()
    geqrf_dtd_untied.last = tp
    return 0


def geqrf_dtd_New(ctx, A, T, window=None):
    return _blocking_New("geqrf_dtd", ctx, lambda: geqrf_dtd(ctx, A, T, window), flops(A.prec, "geqrf", A.m, A.n))


def geqrf_dtd_untied_New(ctx, A, T, window=None):
    return _blocking_New("geqrf_dtd_untied", ctx, lambda: geqrf_dtd_untied(ctx, A, T, window),
                         flops(A.prec, "geqrf", A.m, A.n))


# ----------------------------------------------------------------------------- LU (incremental pivoting)
def _insert_getrf_incpiv(tp, A, L, IPIV, info):
    """zgetrf_incpiv.jdf task classes as DTD tasks (tests/testing_zgetrf_incpiv_dtd.c)."""
    kd = lu_incpiv_ops.kinds(A.dtype, L.mb, A.nb, info)
    tc = {k: tp.task_class(k, kind=kd[k]) for k in ("getrf", "gessm", "tstrf", "ssssm")}
    Tl = dtd.tile_of
    In, InOut, Aff = dtd.INPUT, dtd.INOUT, dtd.AFFINITY
    for k in range(min(A.mt, A.nt)):
        rk, ck = A.tile_rows(k), A.tile_cols(k)
        tp.insert_task(tc["getrf"], (Tl(A, k, k), InOut | Aff), (Tl(IPIV, k, k), InOut), (rk, ck, k * A.nb))
        for n in range(k + 1, A.nt):
            tp.insert_task(tc["gessm"], (Tl(A, k, n), InOut | Aff), (Tl(A, k, k), In), (Tl(IPIV, k, k), In),
                           (rk, A.tile_cols(n), min(rk, ck)))
        for m in range(k + 1, A.mt):
            rm = A.tile_rows(m)
            tp.insert_task(tc["tstrf"], (Tl(A, k, k), InOut), (Tl(A, m, k), InOut | Aff), (Tl(L, m, k), InOut),
                           (Tl(IPIV, m, k), InOut), (rm, ck, k * A.nb))
            for n in range(k + 1, A.nt):
                tp.insert_task(tc["ssssm"], (Tl(A, k, n), InOut), (Tl(A, m, n), InOut | Aff), (Tl(L, m, k), In),
                               (Tl(IPIV, m, k), In), (Tl(A, m, k), In), (rm, A.tile_cols(n), ck))
    tp.data_flush_all(A)
    tp.data_flush_all(L)
    tp.data_flush_all(IPIV)


def getrf_incpiv_dtd(ctx, A, L, IPIV, window=None):
    """Blocking DTD LU with incremental pivoting; returns info (0 = success)."""
    if A.mb != A.nb:
        raise ValueError("square tiles required")
    if L.mb > 32:
        raise ValueError("IB must be <= 32")
    info = torch.zeros(1, dtype=torch.int32, device=A.device)
    tp = dtd.taskpool_new(ctx, "getrf_incpiv_dtd", window=window)
    tp.flops = flops(A.prec, "getrf", A.m, A.n)
    tp.on_complete(_info_reducer(ctx, info))
    _insert_getrf_incpiv(tp, A, L, IPIV, info)
    r = tp.wait()
    getrf_incpiv_dtd.last = tp
    return r


def getrf_incpiv_dtd_New(ctx, A, L, IPIV, window=None):
    return _blocking_New("getrf_incpiv_dtd", ctx, lambda: getrf_incpiv_dtd(ctx, A, L, IPIV, window),
                         flops(A.prec, "getrf", A.m, A.n))
