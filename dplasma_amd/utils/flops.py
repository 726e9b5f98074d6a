"""Floating-point operation counts (LAPACK working-note formulas).

Same formulas as the reference's ``src/flops.h:33-395`` so that GFLOP/s printed
by our harness is comparable with the reference's ``[****] TIME(s) ... gflops``
lines.  ``flops(prec, op, ...)`` returns real flops: fmuls + fadds for real
precisions and 6*fmuls + 2*fadds for complex ones.
"""
from __future__ import annotations


def fmuls_gemm(m, n, k): return float(m) * n * k
def fadds_gemm(m, n, k): return float(m) * n * k
def fmuls_gemv(m, n): return float(m) * n + 2.0 * m
def fadds_gemv(m, n): return float(m) * n
def fmuls_symm(left, m, n): return fmuls_gemm(m, m, n) if left else fmuls_gemm(m, n, n)
fadds_symm = fmuls_symm
def fmuls_syrk(k, n): return 0.5 * k * n * (n + 1.0)
fadds_syrk = fmuls_syrk
def fmuls_syr2k(k, n): return float(k) * n * n
def fadds_syr2k(k, n): return float(k) * n * n + n
def _fmuls_trmm2(m, n): return 0.5 * n * m * (m + 1.0)
def _fadds_trmm2(m, n): return 0.5 * n * m * (m - 1.0)
def fmuls_trmm(left, m, n): return _fmuls_trmm2(m, n) if left else _fmuls_trmm2(n, m)
def fadds_trmm(left, m, n): return _fadds_trmm2(m, n) if left else _fadds_trmm2(n, m)
fmuls_trsm = fmuls_trmm
fadds_trsm = fmuls_trmm  # the reference defines FADDS_TRSM as FMULS_TRMM (flops.h)


def fmuls_getrf(m, n):
    m, n = float(m), float(n)
    if m < n:
        return 0.5 * m * (m * (n - m / 3.0 - 1.0) + n) + 2.0 / 3.0 * m
    return 0.5 * n * (n * (m - n / 3.0 - 1.0) + m) + 2.0 / 3.0 * n


def fadds_getrf(m, n):
    m, n = float(m), float(n)
    if m < n:
        return 0.5 * m * (m * (n - m / 3.0) - n) + m / 6.0
    return 0.5 * n * (n * (m - n / 3.0) - m) + n / 6.0


def fmuls_getrs(n, nrhs): return float(nrhs) * n * n
def fadds_getrs(n, nrhs): return float(nrhs) * n * (n - 1.0)
def fmuls_getri(n): n = float(n); return n * (5.0 / 6.0 + n * (2.0 / 3.0 * n + 0.5))
def fadds_getri(n): n = float(n); return n * (5.0 / 6.0 + n * (2.0 / 3.0 * n - 1.5))
def fmuls_potrf(n): n = float(n); return n * ((n / 6.0 + 0.5) * n + 1.0 / 3.0)
def fadds_potrf(n): n = float(n); return n * ((n / 6.0) * n - 1.0 / 6.0)
def fmuls_potri(n): n = float(n); return n * (2.0 / 3.0 + n * (n / 3.0 + 1.0))
def fadds_potri(n): n = float(n); return n * (1.0 / 6.0 + n * (n / 3.0 - 0.5))
def fmuls_potrs(n, nrhs): return float(nrhs) * n * (n + 1.0)
def fadds_potrs(n, nrhs): return float(nrhs) * n * (n - 1.0)
def fmuls_hetrf(n): n = float(n); return n * ((n / 6.0 + 0.5) * n + 10.0 / 3.0)
def fadds_hetrf(n): n = float(n); return n * ((n / 6.0) * n - 1.0 / 6.0)
def fmuls_trtri(n): n = float(n); return n * (n * (n / 6.0 + 0.5) + 1.0 / 3.0)
def fadds_trtri(n): n = float(n); return n * (n * (n / 6.0 - 0.5) + 1.0 / 3.0)


def fmuls_geqrf(m, n):
    m, n = float(m), float(n)
    if m > n:
        return n * (n * (0.5 - n / 3.0 + m) + m + 23.0 / 6.0)
    return m * (m * (-0.5 - m / 3.0 + n) + 2.0 * n + 23.0 / 6.0)


def fadds_geqrf(m, n):
    m, n = float(m), float(n)
    if m > n:
        return n * (n * (0.5 - n / 3.0 + m) + 5.0 / 6.0)
    return m * (m * (-0.5 - m / 3.0 + n) + n + 5.0 / 6.0)


def fmuls_gelqf(m, n):
    m, n = float(m), float(n)
    if m > n:
        return n * (n * (0.5 - n / 3.0 + m) + m + 29.0 / 6.0)
    return m * (m * (-0.5 - m / 3.0 + n) + 2.0 * n + 29.0 / 6.0)


def fadds_gelqf(m, n):
    m, n = float(m), float(n)
    if m > n:
        return n * (n * (-0.5 - n / 3.0 + m) + m + 5.0 / 6.0)
    return m * (m * (0.5 - m / 3.0 + n) + 5.0 / 6.0)


def fmuls_ungqr(m, n, k):
    m, n, k = float(m), float(n), float(k)
    return k * (2.0 * m * n + 2.0 * n - 5.0 / 3.0 + k * (2.0 / 3.0 * k - (m + n) - 1.0))


def fadds_ungqr(m, n, k):
    m, n, k = float(m), float(n), float(k)
    return k * (2.0 * m * n + n - m + 1.0 / 3.0 + k * (2.0 / 3.0 * k - (m + n)))


def fmuls_unmqr(m, n, k, left=True):
    m, n, k = float(m), float(n), float(k)
    return 2.0 * n * m * k - n * k * k + 2.0 * n * k if left else 2.0 * n * m * k - m * k * k + m * k + n * k - 0.5 * k * k + 0.5 * k


def fadds_unmqr(m, n, k, left=True):
    m, n, k = float(m), float(n), float(k)
    return 2.0 * n * m * k - n * k * k + n * k if left else 2.0 * n * m * k - m * k * k + m * k


def fmuls_geqrs(m, n, nrhs): return float(nrhs) * (n * (2.0 * m - 0.5 * n + 2.5))
def fadds_geqrs(m, n, nrhs): return float(nrhs) * (n * (2.0 * m - 0.5 * n + 0.5))
def fmuls_heev(n): return 2.0 / 3.0 * float(n) ** 3
fadds_heev = fmuls_heev


def fmuls_hetrd(n):
    n = float(n)
    return n * (n * (2.0 / 3.0 * n + 2.5) - 1.0 / 6.0)


def fadds_hetrd(n):
    n = float(n)
    return n * (n * (2.0 / 3.0 * n + 1.0) - 8.0 / 3.0)


def fmuls_gebrd(m, n):
    m, n = float(m), float(n)
    if m < n:
        m, n = n, m
    return n * (n * (2.0 * m - 2.0 / 3.0 * n + 2.0) + 20.0 / 3.0)


def fadds_gebrd(m, n):
    m, n = float(m), float(n)
    if m < n:
        m, n = n, m
    return n * (n * (2.0 * m - 2.0 / 3.0 * n + 1.0) - m + 5.0 / 3.0)


_OPS = {
    "gemm": (fmuls_gemm, fadds_gemm), "gemv": (fmuls_gemv, fadds_gemv),
    "symm": (fmuls_symm, fadds_symm), "hemm": (fmuls_symm, fadds_symm),
    "syrk": (fmuls_syrk, fadds_syrk), "herk": (fmuls_syrk, fadds_syrk),
    "syr2k": (fmuls_syr2k, fadds_syr2k), "her2k": (fmuls_syr2k, fadds_syr2k),
    "trmm": (fmuls_trmm, fadds_trmm), "trsm": (fmuls_trsm, fadds_trsm),
    "getrf": (fmuls_getrf, fadds_getrf), "getrs": (fmuls_getrs, fadds_getrs), "getri": (fmuls_getri, fadds_getri),
    "potrf": (fmuls_potrf, fadds_potrf), "potri": (fmuls_potri, fadds_potri), "potrs": (fmuls_potrs, fadds_potrs),
    "hetrf": (fmuls_hetrf, fadds_hetrf), "sytrf": (fmuls_hetrf, fadds_hetrf),
    "trtri": (fmuls_trtri, fadds_trtri), "lauum": (lambda n: fmuls_potri(n) - fmuls_trtri(n), lambda n: fadds_potri(n) - fadds_trtri(n)),
    "geqrf": (fmuls_geqrf, fadds_geqrf), "gelqf": (fmuls_gelqf, fadds_gelqf),
    "ungqr": (fmuls_ungqr, fadds_ungqr), "unglq": (fmuls_ungqr, fadds_ungqr),
    "unmqr": (fmuls_unmqr, fadds_unmqr), "unmlq": (fmuls_unmqr, fadds_unmqr),
    "geqrs": (fmuls_geqrs, fadds_geqrs), "heev": (fmuls_heev, fadds_heev),
    "hetrd": (fmuls_hetrd, fadds_hetrd), "herbt": (fmuls_hetrd, fadds_hetrd), "gebrd": (fmuls_gebrd, fadds_gebrd),
}


def flops(prec: str, op: str, *args) -> float:
    """Real flop count for ``op`` in precision ``prec`` ('s','d','c','z')."""
    fm, fa = _OPS[op]
    m, a = fm(*args), fa(*args)
    return 6.0 * m + 2.0 * a if prec in ("c", "z") else m + a
