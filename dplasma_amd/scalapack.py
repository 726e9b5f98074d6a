"""ScaLAPACK-compatible entry points (p?gemm_, p?potrf_, p?getrf_, p?trsm_, p?trmm_, p?latsqr_).

Reference: ``src/scalapack_wrappers/`` (``dplasma_wrapper_pd*.c``, descriptor
unpacking ``common.h:237-262``, ``GENERATE_F77_BINDINGS``), which let a
ScaLAPACK program call DPLASMA on its own block-cyclic arrays.

A ScaLAPACK array descriptor is ``[dtype, ctxt, m, n, mb, nb, rsrc, csrc, lld]``
and the local array is column-major with leading dimension ``lld``, blocks
stored contiguously by local block index -- exactly dplasma_amd's LAPACK
storage, so the shims wrap the caller's local array (a torch tensor, on the
GPU or the host) as a :class:`TiledMatrix` without copying (``rsrc/csrc`` map
to the grid offsets ``ip/jq``).  ``ia, ja`` (1-based) select a sub-matrix; a
non tile-aligned one is staged through an aligned copy.  BLACS contexts are
handles onto dplasma_amd contexts (``blacs_gridinit``).
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch

from .constants import (STORAGE_LAPACK, dplasmaConjTrans, dplasmaLeft, dplasmaLower, dplasmaNoTrans,
                        dplasmaNonUnit, dplasmaRight, dplasmaTrans, dplasmaUnit, dplasmaUpper)
from .descriptor import TiledMatrix

DTYPE_, CTXT_, M_, N_, MB_, NB_, RSRC_, CSRC_, LLD_ = range(9)
_CTXTS: Dict[int, object] = {}

_CH = {"N": dplasmaNoTrans, "T": dplasmaTrans, "C": dplasmaConjTrans, "L": dplasmaLower, "U": dplasmaUpper,
       "R": dplasmaRight, "S": dplasmaLeft}
_SIDE = {"L": dplasmaLeft, "R": dplasmaRight}
_DIAG = {"N": dplasmaNonUnit, "U": dplasmaUnit}
PREC_DTYPE = {"s": torch.float32, "d": torch.float64, "c": torch.complex64, "z": torch.complex128}


def blacs_gridinit(ctx, P=None, Q=None) -> int:
    """Register a dplasma_amd context as a BLACS context handle (grid P x Q of ctx)."""
    h = len(_CTXTS) + 1
    _CTXTS[h] = ctx
    return h


def blacs_gridinfo(ictxt):
    ctx = _CTXTS[ictxt]
    return ctx.P, ctx.Q, ctx.rank // ctx.Q, ctx.rank % ctx.Q


def numroc(n, nb, iproc, isrcproc, nprocs) -> int:
    """Number of rows/cols of a block-cyclic dimension owned by iproc (ScaLAPACK NUMROC)."""
    mydist = (nprocs + iproc - isrcproc) % nprocs
    nblocks = n // nb
    num = (nblocks // nprocs) * nb
    extra = nblocks % nprocs
    if mydist < extra:
        num += nb
    elif mydist == extra:
        num += n % nb
    return num


def descinit(m, n, mb, nb, rsrc, csrc, ictxt, lld):
    return [1, ictxt, m, n, mb, nb, rsrc, csrc, lld]


def _wrap(a, desc, dtype):
    ctx = _CTXTS[desc[CTXT_]]
    flat = a.reshape(-1) if a.is_contiguous() else a.t().reshape(-1)
    M = TiledMatrix(dtype, desc[MB_], desc[NB_], desc[M_], desc[N_], P=ctx.P, Q=ctx.Q, ip=desc[RSRC_],
                    jq=desc[CSRC_], rank=ctx.rank, device=flat.device, storage=STORAGE_LAPACK, lld=desc[LLD_],
                    data=flat, name="scalapack")
    return ctx, M


def _sub(ctx, M, ia, ja, m, n):
    """Sub-matrix (1-based ia, ja) of M; returns (view, writeback callable)."""
    i, j = ia - 1, ja - 1
    if i % M.mb == 0 and j % M.nb == 0:
        return M.submatrix(i, j, m, n), (lambda: None)
    from .models.redistribute import redistribute
    T = TiledMatrix(M.dtype, M.mb, M.nb, m, n, P=M.grid.P, Q=M.grid.Q, rank=M.rank, device=M.device,
                    storage=STORAGE_LAPACK, name="stage")
    redistribute(ctx, M, T, m, n, i, j, 0, 0)
    return T, (lambda: redistribute(ctx, T, M, m, n, 0, 0, i, j))


def _make(prec):
    dt = PREC_DTYPE[prec]

    def pgemm_(transa, transb, m, n, k, alpha, a, ia, ja, desca, b, ib, jb, descb, beta, c, ic, jc, descc):
        from .models.gemm import gemm
        ctx, A = _wrap(a, desca, dt)
        _, B = _wrap(b, descb, dt)
        _, C = _wrap(c, descc, dt)
        ta, tb = _CH[transa.upper()], _CH[transb.upper()]
        Asub, _ = _sub(ctx, A, ia, ja, *((m, k) if ta == dplasmaNoTrans else (k, m)))
        Bsub, _ = _sub(ctx, B, ib, jb, *((k, n) if tb == dplasmaNoTrans else (n, k)))
        Csub, wb = _sub(ctx, C, ic, jc, m, n)
        gemm(ctx, ta, tb, alpha, Asub, Bsub, beta, Csub)
        wb()

    def ppotrf_(uplo, n, a, ia, ja, desca):
        from .models.potrf import potrf
        ctx, A = _wrap(a, desca, dt)
        Asub, wb = _sub(ctx, A, ia, ja, n, n)
        info = potrf(ctx, _CH[uplo.upper()], Asub)
        wb()
        return info

    def pgetrf_(m, n, a, ia, ja, desca, ipiv=None):
        """LU with partial pivoting; ipiv (local int32, LOCr(m)+mb) gets global 1-based pivots of local rows."""
        from .models.lu import getrf_ptgpanel, ptgpanel_ipiv_descriptor, _gather_ipiv
        ctx, A = _wrap(a, desca, dt)
        Asub, wb = _sub(ctx, A, ia, ja, m, n)
        IP = ptgpanel_ipiv_descriptor(ctx, Asub)
        info = getrf_ptgpanel(ctx, Asub, IP)
        wb()
        if ipiv is not None:
            piv = _gather_ipiv(ctx, IP)
            l = 0
            for t in Asub.rows:
                for r in range(Asub._grows(t)):
                    g = t * Asub.mb + r
                    if g < len(piv) and l < len(ipiv):
                        ipiv[l] = int(piv[g]) + ia - 1
                    l += 1
        return info

    def ptrsm_(side, uplo, transa, diag, m, n, alpha, a, ia, ja, desca, b, ib, jb, descb):
        from .models.blas3 import trsm
        ctx, A = _wrap(a, desca, dt)
        _, B = _wrap(b, descb, dt)
        k = m if side.upper() == "L" else n
        Asub, _ = _sub(ctx, A, ia, ja, k, k)
        Bsub, wb = _sub(ctx, B, ib, jb, m, n)
        trsm(ctx, _SIDE[side.upper()], _CH[uplo.upper()], _CH[transa.upper()], _DIAG[diag.upper()], alpha,
             Asub, Bsub)
        wb()

    def ptrmm_(side, uplo, transa, diag, m, n, alpha, a, ia, ja, desca, b, ib, jb, descb):
        from .models.blas3 import trmm
        ctx, A = _wrap(a, desca, dt)
        _, B = _wrap(b, descb, dt)
        k = m if side.upper() == "L" else n
        Asub, _ = _sub(ctx, A, ia, ja, k, k)
        Bsub, wb = _sub(ctx, B, ib, jb, m, n)
        trmm(ctx, _SIDE[side.upper()], _CH[uplo.upper()], _CH[transa.upper()], _DIAG[diag.upper()], alpha,
             Asub, Bsub)
        wb()

    def platsqr_(m, n, a, ia, ja, desca, tau=None, ib=None):
        """Tall-skinny QR of A(ia:, ja:) in place (tile Householder QR, hierarchical tree over the
        process rows, as dplasma_wrapper_pdlatsqr.c runs dgeqrf on the caller's array).  R is left in
        the upper triangle; the reflectors use the tile layout (not LAPACK's), and ``tau`` receives
        the T diagonal of the diagonal tiles.  Returns (info, TS, TT, tree) so Q can be applied."""
        from .models import qr, qrtree
        ctx, A = _wrap(a, desca, dt)
        Asub, wb = _sub(ctx, A, ia, ja, m, n)
        ibv = ib or min(32, Asub.nb)
        TS = TiledMatrix(dt, ibv, Asub.nb, Asub.mt * ibv, Asub.nt * Asub.nb, P=ctx.P, Q=ctx.Q, rank=ctx.rank,
                         device=Asub.device)
        TT = TiledMatrix(dt, ibv, Asub.nb, Asub.mt * ibv, Asub.nt * Asub.nb, P=ctx.P, Q=ctx.Q, rank=ctx.rank,
                         device=Asub.device)
        tree = qrtree.hqr_init(dplasmaNoTrans, Asub, qrtree.GREEDY_TREE, qrtree.GREEDY_TREE, 4, ctx.P)
        qr.geqrf_param(ctx, tree, Asub, TS, TT)
        wb()
        if tau is not None:
            vals = torch.zeros(min(m, n), dtype=dt)
            for (i, j) in TS.local_tiles():
                if i == j and i < Asub.mt:
                    t = TS.tile(i, j).cpu()
                    for c in range(t.shape[1]):
                        g = j * Asub.nb + c
                        if g < len(vals):
                            vals[g] = t[c % ibv, c]
            if ctx.world > 1:
                import torch.distributed as dist
                v = vals.to(Asub.device)
                dist.all_reduce(v)
                vals = v.cpu()
            tau[: len(vals)] = vals.to(tau.device)
        return 0, TS, TT, tree

    return {"gemm_": pgemm_, "potrf_": ppotrf_, "getrf_": pgetrf_, "trsm_": ptrsm_, "trmm_": ptrmm_,
            "latsqr_": platsqr_}


for _p in "sdcz":
    for _name, _fn in _make(_p).items():
        globals()["p" + _p + _name] = _fn

__all__ = ["blacs_gridinit", "blacs_gridinfo", "numroc", "descinit"] + \
    ["p" + p + n for p in "sdcz" for n in ("gemm_", "potrf_", "getrf_", "trsm_", "trmm_", "latsqr_")]
