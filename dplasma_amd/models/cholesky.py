"""Cholesky-based drivers: POTRS, POSV, TRTRI, LAUUM, POTRI, POINV.

Reference: ``src/zpotrs_wrapper.c`` / ``zposv_wrapper.c`` (potrf + 2 trsm),
``src/ztrtri_L.jdf`` / ``ztrtri_U.jdf`` (task classes trtri_ztrsmR, trtri_zgemm,
trtri_ztrsmL, trtri_ztrtri, :22-169), ``src/zlauum_L.jdf`` (lauum_zherk,
lauum_zgemm, lauum_ztrmm, lauum_zlauum, :42-147), ``src/zpotri_wrapper.c``
(trtri + lauum) and ``src/zpoinv_L.jdf`` (the 12 task classes of potrf + trtri
+ lauum in one DAG; here the three programs are queued back to back, each one
batched per step).
"""
from __future__ import annotations

from ..constants import (dplasmaConjTrans, dplasmaLeft, dplasmaLower, dplasmaNoTrans, dplasmaNonUnit, dplasmaRight,
                         dplasmaUpper)
from ..ops import tile_ops as ops
from ..ops.batch import MASK_LOWER, MASK_UPPER
from ..runtime.taskpool import Taskpool
from ..runtime.tileprog import TileProgram
from ..utils.flops import flops
from . import blas3
from .potrf import potrf_New

N_, C_ = dplasmaNoTrans, dplasmaConjTrans


class _Seq(Taskpool):
    """A taskpool that runs several taskpools back to back (parsec_compose analogue)."""

    def __init__(self, name, ctx, parts, result_from=0):
        super().__init__(name, ctx)
        self.parts = parts
        self.flops = sum(p.flops for p in parts)
        self._rf = result_from

    def run(self, ctx=None):
        import time
        self._t_run = time.perf_counter()
        for i, p in enumerate(self.parts):
            p.run(ctx or self.ctx)
            if i < len(self.parts) - 1:
                p.complete(ctx or self.ctx)

    def complete(self, ctx=None):
        r = self.parts[-1].complete(ctx or self.ctx)
        res = self.parts[self._rf]._result if self._rf < len(self.parts) - 1 else r
        for fn in self._on_complete:
            v = fn()
            if v is not None:
                res = v
        self._result = res
        return res

    def destruct(self):
        for p in self.parts:
            p.destruct()


def compose(ctx, *tps, name="compose"):
    """Chain taskpools (``parsec_compose``, used by the reference's zheev, src/zheev_wrapper.c:100)."""
    return _Seq(name, ctx, list(tps))


# ----------------------------------------------------------------------------- POTRS / POSV
def potrs_New(ctx, uplo, A, B):
    if uplo == dplasmaLower:
        prog = blas3.trsm_program(ctx, dplasmaLeft, dplasmaLower, N_, dplasmaNonUnit, 1.0, A, B, name="potrs")
        blas3.trsm_program(ctx, dplasmaLeft, dplasmaLower, C_, dplasmaNonUnit, 1.0, A, B, prog=prog)
    else:
        prog = blas3.trsm_program(ctx, dplasmaLeft, dplasmaUpper, C_, dplasmaNonUnit, 1.0, A, B, name="potrs")
        blas3.trsm_program(ctx, dplasmaLeft, dplasmaUpper, N_, dplasmaNonUnit, 1.0, A, B, prog=prog)
    prog.flops = flops(A.prec, "potrs", A.n, B.n)
    return prog.compile()


def potrs(ctx, uplo, A, B):
    return potrs_New(ctx, uplo, A, B).execute(ctx)


def posv_New(ctx, uplo, A, B):
    return _Seq("posv", ctx, [potrf_New(ctx, uplo, A), potrs_New(ctx, uplo, A, B)], result_from=0)


def posv(ctx, uplo, A, B):
    """Solve A X = B with A SPD (A overwritten by its factor, B by X); returns potrf info."""
    tp1 = potrf_New(ctx, uplo, A)
    info = tp1.execute(ctx)
    if info != 0:
        return info
    potrs(ctx, uplo, A, B)
    return 0


# ----------------------------------------------------------------------------- TRTRI
def _tile_op_trtri(uplo, diag, A, key):
    def fn(res):
        base, off, ld = res[key]
        ops.trtri_tile(uplo, diag, base, off, A.tile_rows(key[1]), ld)
    return fn


def _tile_op_lauum(uplo, A, key):
    def fn(res):
        base, off, ld = res[key]
        ops.lauum_tile(uplo, base, off, A.tile_rows(key[1]), ld)
    return fn


def trtri_program(ctx, uplo, diag, A, prog=None):
    prog = prog or TileProgram(ctx, "trtri")
    prog.flops += flops(A.prec, "trtri", A.n)
    nt = A.nt
    lower = uplo == dplasmaLower
    for k in range(nt):
        s = prog.stage(f"trtri_trsmR({k})")
        if lower:
            for m in range(k + 1, nt):
                s.trsm(dplasmaRight, uplo, N_, diag, -1.0, (A, k, k), (A, m, k))
        else:
            for n in range(k + 1, nt):
                s.trsm(dplasmaLeft, uplo, N_, diag, -1.0, (A, k, k), (A, k, n))
        s = prog.stage(f"trtri_gemm({k})")
        if lower:
            for m in range(k + 1, nt):
                for n in range(k):
                    s.gemm((A, m, n), [((A, m, k), N_, (A, k, n), N_)], alpha=1.0, beta=1.0)
        else:
            for m in range(k):
                for n in range(k + 1, nt):
                    s.gemm((A, m, n), [((A, m, k), N_, (A, k, n), N_)], alpha=1.0, beta=1.0)
        s = prog.stage(f"trtri_trsmL({k})")
        if lower:
            for n in range(k):
                s.trsm(dplasmaLeft, uplo, N_, diag, 1.0, (A, k, k), (A, k, n))
        else:
            for m in range(k):
                s.trsm(dplasmaRight, uplo, N_, diag, 1.0, (A, k, k), (A, m, k))
        s = prog.stage(f"trtri_trtri({k})")
        key = (prog.mid(A), k, k)
        s.batch_fn([(A, k, k)], [], _tile_op_trtri(uplo, diag, A, key))
    return prog


def trtri_New(ctx, uplo, diag, A):
    return trtri_program(ctx, uplo, diag, A).compile()


def trtri(ctx, uplo, diag, A):
    return trtri_New(ctx, uplo, diag, A).execute(ctx)


# ----------------------------------------------------------------------------- LAUUM
def lauum_program(ctx, uplo, A, prog=None):
    """A := L^H L (lower) or U U^H (upper), in the uplo triangle."""
    prog = prog or TileProgram(ctx, "lauum")
    prog.flops += flops(A.prec, "lauum", A.n)
    nt = A.nt
    lower = uplo == dplasmaLower
    Tri = A.like(name="Ltri")
    W = A.like(name="W")
    prog._keep = getattr(prog, "_keep", ()) + (Tri, W)
    for k in range(nt):
        s = prog.stage(f"lauum_herk_gemm({k})")
        for m in range(k):
            for n in range(m + 1):
                if lower:   # A(m,n) += A(k,m)^H A(k,n)
                    s.gemm((A, m, n), [((A, k, m), C_, (A, k, n), N_)], beta=1.0,
                           mask=MASK_LOWER if m == n else 0)
                else:       # A(n,m) += A(n,k) A(m,k)^H  (upper: U U^H)
                    s.gemm((A, n, m), [((A, n, k), N_, (A, m, k), C_)], beta=1.0,
                           mask=MASK_UPPER if m == n else 0)
        # trmm of the off-diagonal block row/col with the (original) diagonal tile
        s = prog.stage(f"lauum_tri({k})")
        s.laset((Tri, k, k), 0, 0.0, 0.0)
        s = prog.stage(f"lauum_tricopy({k})")
        s.copy((A, k, k), (Tri, k, k), part=1 if lower else 2)
        s = prog.stage(f"lauum_trmm({k})")
        for n in range(k):
            if lower:   # W(k,n) = A(k,k)^H A(k,n)
                s.gemm((W, k, n), [((Tri, k, k), C_, (A, k, n), N_)], beta=0.0)
            else:       # W(n,k) = A(n,k) A(k,k)^H
                s.gemm((W, n, k), [((A, n, k), N_, (Tri, k, k), C_)], beta=0.0)
        s = prog.stage(f"lauum_copyback({k})")
        for n in range(k):
            if lower:
                s.copy((W, k, n), (A, k, n))
            else:
                s.copy((W, n, k), (A, n, k))
        s = prog.stage(f"lauum_lauum({k})")
        key = (prog.mid(A), k, k)
        s.batch_fn([(A, k, k)], [], _tile_op_lauum(uplo, A, key))
    return prog


def lauum_New(ctx, uplo, A):
    prog = lauum_program(ctx, uplo, A)
    tp = prog.compile()
    tp._keep = prog._keep
    return tp


def lauum(ctx, uplo, A):
    return lauum_New(ctx, uplo, A).execute(ctx)


# ----------------------------------------------------------------------------- POTRI / POINV
def potri_New(ctx, uplo, A):
    prog = trtri_program(ctx, uplo, dplasmaNonUnit, A, prog=TileProgram(ctx, "potri"))
    lauum_program(ctx, uplo, A, prog=prog)
    tp = prog.compile()
    tp._keep = prog._keep
    return tp


def potri(ctx, uplo, A):
    """Inverse of an SPD matrix from its Cholesky factor (in place)."""
    return potri_New(ctx, uplo, A).execute(ctx)


def poinv_New(ctx, uplo, A):
    return _Seq("poinv", ctx, [potrf_New(ctx, uplo, A), potri_New(ctx, uplo, A)], result_from=0)


def poinv(ctx, uplo, A):
    """A := inv(A) for SPD A (potrf + trtri + lauum); returns the potrf info."""
    info = potrf_New(ctx, uplo, A).execute(ctx)
    if info != 0:
        return info
    potri(ctx, uplo, A)
    return 0
