"""LU incremental-pivoting tile kernels as DAG kinds (GPU launch + CPU reference).

GPU: ``csrc/kernels/lu_incpiv.hip``.  CPU: PyTorch transcriptions of the same
algorithms (PLASMA ``CORE_zgetrf_incpiv``, ``CORE_zgessm``, ``CORE_ztstrf``
core_ztstrf.c:100-240, ``CORE_zssssm``), so that the L / IPIV contents are
interchangeable between the two paths.
"""
from __future__ import annotations

import torch

from ..runtime.dag import Kind, R, RW
from . import _lib


def _v(ref, rows, cols):
    base, off, ld = ref
    return torch.as_strided(base, (rows, cols), (1, ld), off)


def _abs1(x):
    return (x.real.abs() + x.imag.abs()) if x.is_complex() else x.abs()


def ref_getrf(A, ipiv, info, base):
    """Partial-pivoting LU of the tile view A (in place), 1-based ipiv."""
    m, n = A.shape
    for j in range(min(m, n)):
        p = j + int(torch.argmax(_abs1(A[j:, j])))
        if p != j:
            A[[j, p], :] = A[[p, j], :]
        ipiv[j] = p + 1
        d = A[j, j]
        if d == 0:
            if info is not None and int(info[0]) == 0:
                info[0] = base + j + 1
            continue
        A[j + 1:, j] /= d
        if j + 1 < n:
            A[j + 1:, j + 1:] -= torch.outer(A[j + 1:, j], A[j, j + 1:])


def ref_gessm(C, LU, ipiv, kk):
    m = C.shape[0]
    for i in range(kk):
        p = int(ipiv[i]) - 1
        if p != i:
            C[[i, p], :] = C[[p, i], :]
    for i in range(kk):
        if i + 1 < m:
            C[i + 1:, :] -= torch.outer(LU[i + 1:m, i], C[i, :])


def ref_ssssm(A1, A2, L1, ipiv, L2, ib, NB, K):
    for ii in range(0, K, ib):
        sb = min(ib, K - ii)
        for i in range(sb):
            im = int(ipiv[ii + i]) - 1
            if im != ii + i:
                r2 = im - NB
                t = A1[ii + i, :].clone()
                A1[ii + i, :] = A2[r2, :]
                A2[r2, :] = t
        for i in range(1, sb):
            A1[ii + i, :] -= L1[i, ii:ii + i] @ A1[ii:ii + i, :]
        A2 -= L2[:, ii:ii + sb] @ A1[ii:ii + sb, :]


def ref_tstrf(U, A, L, ipiv, ib, NB, info, base):
    m, n = A.shape
    L.zero_()
    W = torch.zeros(m, ib, dtype=A.dtype)
    for ii in range(0, n, ib):
        sb = min(n - ii, ib)
        for i in range(sb):
            col = ii + i
            im = int(torch.argmax(_abs1(A[:, col])))
            ipiv[col] = col + 1
            if abs(complex(A[im, col])) > abs(complex(U[col, col])):
                t = L[i, ii:ii + i].clone()
                L[i, ii:ii + i] = W[im, :i]
                W[im, :i] = t
                t = U[col, col:ii + sb].clone()
                U[col, col:ii + sb] = A[im, col:ii + sb]
                A[im, col:ii + sb] = t
                ipiv[col] = NB + im + 1
                A[im, ii:col] = 0
            if info is not None and int(info[0]) == 0 and U[col, col] == 0:
                info[0] = base + col + 1
            u = U[col, col]
            alpha = 0 if u == 0 else 1.0 / u
            A[:, col] *= alpha
            W[:, i] = A[:, col]
            if i + 1 < sb:
                A[:, col + 1:ii + sb] -= torch.outer(A[:, col], U[col, col + 1:ii + sb])
        if ii + sb < n:
            c0 = ii + sb
            for i in range(sb):
                p = int(ipiv[ii + i]) - 1
                if p != ii + i:
                    r2 = p - NB
                    t = U[ii + i, c0:].clone()
                    U[ii + i, c0:] = A[r2, c0:]
                    A[r2, c0:] = t
            for i in range(1, sb):
                U[ii + i, c0:] -= L[i, ii:ii + i] @ U[ii:ii + i, c0:]
            A[:, c0:] -= A[:, ii:ii + sb] @ U[ii:ii + sb, c0:]


def kinds(dtype: torch.dtype, ib: int, NB: int, info: torch.Tensor):
    """Kind set for one call (the info counter is bound into the launchers)."""
    prec = _lib.prec_code(dtype)
    tag = f"_{prec}_{ib}_{NB}_{id(info)}"
    out = {}

    def info_ptr():
        return info.data_ptr() if info is not None and info.is_cuda else None

    def g_getrf(items, n, stream, emax):
        _lib.check(_lib.load().dpl_getrf_tile(prec, n, items, info_ptr(), stream), "getrf_tile")

    def c_getrf(refs, ext):
        m, n, base = ext
        ipiv = refs[1][0][refs[1][1]:refs[1][1] + min(m, n)]
        ref_getrf(_v(refs[0], m, n), ipiv, info, base)
    out["getrf"] = Kind("incpiv_getrf" + tag, (("A", RW, 1), ("IPIV", RW, 3)), 0, g_getrf, c_getrf)

    def g_gessm(items, n, stream, emax):
        _lib.check(_lib.load().dpl_gessm(prec, n, items, emax[1], stream), "gessm")

    def c_gessm(refs, ext):
        m, n, kk = ext
        ipiv = refs[2][0][refs[2][1]:refs[2][1] + kk]
        ref_gessm(_v(refs[0], m, n), _v(refs[1], m, kk), ipiv, kk)
    out["gessm"] = Kind("incpiv_gessm" + tag, (("C", RW, 1), ("LU", R, 2), ("IPIV", R, 3)), 0, g_gessm, c_gessm,
                        prio=1)

    def g_tstrf(items, n, stream, emax):
        _lib.check(_lib.load().dpl_tstrf(prec, n, items, ib, NB, emax[0], info_ptr(), stream), "tstrf")

    def c_tstrf(refs, ext):
        m, n, base = ext
        ipiv = refs[3][0][refs[3][1]:refs[3][1] + n]
        ref_tstrf(_v(refs[0], n, n), _v(refs[1], m, n), _v(refs[2], ib, n), ipiv, ib, NB, info, base)
    out["tstrf"] = Kind("incpiv_tstrf" + tag, (("U", RW, 0), ("A", RW, 1), ("L", RW, 2), ("IPIV", RW, 3)), 1,
                        g_tstrf, c_tstrf)

    def g_ssssm(items, n, stream, emax):
        _lib.check(_lib.load().dpl_ssssm(prec, n, items, emax[1], ib, NB, stream), "ssssm")

    def c_ssssm(refs, ext):
        m, n, K = ext
        ipiv = refs[3][0][refs[3][1]:refs[3][1] + K]
        ref_ssssm(_v(refs[0], K, n), _v(refs[1], m, n), _v(refs[2], ib, K), ipiv, _v(refs[4], m, K), ib, NB, K)
    out["ssssm"] = Kind("incpiv_ssssm" + tag, (("A1", RW, 0), ("A2", RW, 1), ("L1", R, 2), ("IPIV", R, 3),
                                              ("L2", R, 4)), 1, g_ssssm, c_ssssm, prio=1)
    return out
