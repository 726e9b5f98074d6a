"""Numerical verification routines (the reference's ``src/dplasma_zcheck.c``).

All checks run distributed with the library's own kernels (lacpy / laset /
GEMM engine / norms), so a passing check also exercises the native path.

* ``check_potrf``: ||A0 - L L^H|| / (||A0|| N eps)  (or U^H U), threshold 60.
* ``check_axmb``:  ||A x - b|| / ((||A|| ||x|| + ||b||) N eps), threshold 60.
* ``check_gemm``-style comparisons are done in the tests against a dense
  PyTorch fp64 reference.
"""
from __future__ import annotations

import torch

from ..constants import (dplasmaConjTrans, dplasmaInfNorm, dplasmaLower, dplasmaNoTrans, dplasmaUpper,
                         dplasmaUpperLower)
from . import aux
from .gemm import gemm

THRESHOLD = 60.0


def eps_of(dtype) -> float:
    return float(torch.finfo(dtype).eps) / 2.0 if dtype in (torch.float32, torch.complex64) else float(
        torch.finfo(torch.float64).eps) / 2.0


def _eps(A):
    real = torch.float32 if A.dtype in (torch.float32, torch.complex64) else torch.float64
    return float(torch.finfo(real).eps)


def check_potrf(ctx, uplo, A, A0, verbose=False):
    """A holds the factor, A0 the original (full storage, only uplo referenced). Returns (ok, residual)."""
    n = A.n
    Lm = A.like(name="L")
    aux.laset(ctx, dplasmaUpperLower, 0.0, 0.0, Lm)
    aux.lacpy(ctx, uplo, A, Lm)
    R = A0.like(name="R")
    # R = full Hermitian A0 from its uplo triangle
    aux.lacpy(ctx, uplo, A0, R)
    _herm_fill(ctx, uplo, R)
    if uplo == dplasmaLower:
        gemm(ctx, dplasmaNoTrans, dplasmaConjTrans, -1.0, Lm, Lm, 1.0, R)
    else:
        gemm(ctx, dplasmaConjTrans, dplasmaNoTrans, -1.0, Lm, Lm, 1.0, R)
    rn = aux.lange(ctx, dplasmaInfNorm, R)
    an = aux.lanhe(ctx, dplasmaInfNorm, uplo, A0)
    res = rn / (an * n * _eps(A)) if an > 0 else rn
    ok = res < THRESHOLD and res == res
    if verbose and ctx.rank == 0:
        print(f"-- ||L'L-A||_oo/(||A||_oo.N.eps) = {res:e} : {'SUCCESS' if ok else 'FAILED'}")
    return ok, res


def _herm_fill(ctx, uplo, R):
    """Make R Hermitian from its uplo triangle (R := tri(R) + tri(R)^H - diag)."""
    T = R.like(name="T")
    aux.laset(ctx, dplasmaUpperLower, 0.0, 0.0, T)
    aux.geadd_New(ctx, dplasmaConjTrans, 1.0, R, 0.0, T).execute(ctx)  # T = R^H (full)
    # keep the strictly-opposite triangle of T into R
    other = dplasmaUpper if uplo == dplasmaLower else dplasmaLower
    # zero diag of T so only the strict part is copied
    tb = aux.local_tile_batch(T)
    from ..ops import tile_ops as ops
    ops.laset(5, 0.0, 0.0, T.data, T.ld, tb)  # part 5 = diagonal only
    if ctx.is_gpu:
        torch.cuda.synchronize()
    aux.geadd_New(ctx, dplasmaNoTrans, 1.0, T, 1.0, R, uplo=other).execute(ctx)


def check_axmb(ctx, A, X, B, verbose=False):
    """||A x - b||_oo / ((||A||_oo ||x||_oo + ||b||_oo) N eps)."""
    an = aux.lange(ctx, dplasmaInfNorm, A)
    xn = aux.lange(ctx, dplasmaInfNorm, X)
    bn = aux.lange(ctx, dplasmaInfNorm, B)
    R = B.like(name="R")
    aux.lacpy(ctx, dplasmaUpperLower, B, R)
    gemm(ctx, dplasmaNoTrans, dplasmaNoTrans, -1.0, A, X, 1.0, R)
    rn = aux.lange(ctx, dplasmaInfNorm, R)
    res = rn / ((an * xn + bn) * A.n * _eps(A))
    ok = res < THRESHOLD and res == res
    if verbose and ctx.rank == 0:
        print(f"-- ||Ax-B||_oo/((||A||_oo||x||_oo+||B||_oo).N.eps) = {res:e} : {'SUCCESS' if ok else 'FAILED'}")
    return ok, res
