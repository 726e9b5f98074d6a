"""Householder QR/LQ tile kernels as DAG kinds (GPU launch + CPU reference).

GPU: ``csrc/kernels/qr.hip`` (one batched launch per level).  CPU: a direct
PyTorch transcription of the same math, used on hosts without a GPU and as
the numerics reference in tests.

Semantics follow PLASMA's core_blas routines used by the reference
(``CORE_zgeqrt`` core_zgeqrt.c:86, ``CORE_zunmqr`` core_zunmqr.c:108,
``CORE_ztsqrt`` core_ztsqrt.c:97, ``CORE_ztsmqr`` core_ztsmqr.c:124,
``CORE_zttqrt``/``CORE_zttmqr``): Householder vectors are stored in place of
the annihilated entries, and T holds, for every IB-wide block of reflectors,
the upper-triangular factor of the compact-WY form H = I - V T V^H in an
IB x NB tile.  LQ kernels (``CORE_zgelqt``, ``CORE_ztslqt``, ``CORE_ztsmlq``,
``CORE_zunmlq``, ...) are the QR kernels applied to conjugate-transposed tile
views (``tr=1, cj=1``): LQ of A is QR of A^H.
"""
from __future__ import annotations

import math
from functools import lru_cache

import torch

from ..runtime.dag import Kind, R, RW
from . import _lib


# ----------------------------------------------------------------------------- views (CPU)
def _load(ref, rows, cols, tr, cj):
    base, off, ld = ref
    st = (ld, 1) if tr else (1, ld)
    v = torch.as_strided(base, (rows, cols), st, off)
    x = v.clone()
    return x.conj().resolve_conj() if (cj and x.is_complex()) else x


def _store(ref, x, tr, cj, mask=None):
    base, off, ld = ref
    rows, cols = x.shape
    st = (ld, 1) if tr else (1, ld)
    v = torch.as_strided(base, (rows, cols), st, off)
    y = x.conj().resolve_conj() if (cj and x.is_complex()) else x
    if mask is None:
        v.copy_(y)
    else:
        v.copy_(torch.where(mask, y, v))


def _larfg(alpha, x):
    """(beta, tau, scale) of the Householder reflector annihilating x below alpha (zlarfg)."""
    xn2 = float((x.abs() ** 2).sum()) if x.numel() else 0.0
    a = complex(alpha)
    ar, ai = a.real, a.imag
    if xn2 == 0.0 and ai == 0.0:
        return alpha, 0.0, 0.0
    nrm = math.sqrt(ar * ar + ai * ai + xn2)
    beta = -nrm if ar >= 0 else nrm
    tau = complex((beta - ar) / beta, -ai / beta)
    scal = 1.0 / (a - beta)
    if not x.is_complex():
        return beta, tau.real, scal.real
    return beta, tau, scal


def _cj(z):
    return z.conjugate() if isinstance(z, complex) else z


def _ref_geqrt(A, T, ib):
    """In-place QR of A (m x n); T (>= ib rows, n cols) gets the block T factors."""
    m, n = A.shape
    k = min(m, n)
    for i0 in range(0, k, ib):
        sb = min(ib, k - i0)
        taus = []
        for j in range(i0, i0 + sb):
            beta, tau, scal = _larfg(A[j, j].item(), A[j + 1:, j])
            A[j + 1:, j] *= scal
            A[j, j] = beta
            taus.append(tau)
            c1 = i0 + sb
            if j + 1 < c1:
                v = torch.cat([torch.ones(1, dtype=A.dtype), A[j + 1:, j]])
                w = v.conj() @ A[j:, j + 1:c1]
                A[j:, j + 1:c1] -= _cj(tau) * torch.outer(v, w)
        V = torch.tril(A[i0:, i0:i0 + sb], -1)
        V[:sb, :sb] += torch.eye(sb, dtype=A.dtype)
        Tb = _larft(V, taus)
        T[:sb, i0:i0 + sb] = Tb
        if i0 + sb < n:
            C = A[i0:, i0 + sb:]
            C -= V @ (Tb.conj().T @ (V.conj().T @ C))


def _larft(V, taus):
    sb = len(taus)
    Tb = torch.zeros(sb, sb, dtype=V.dtype)
    for j in range(sb):
        Tb[j, j] = taus[j]
        if j:
            y = V[:, :j].conj().T @ V[:, j]
            Tb[:j, j] = -taus[j] * (Tb[:j, :j] @ y)
    return Tb


def _ref_unmqr(C, V, T, ib, k, conjtrans):
    m = C.shape[0]
    blocks = list(range(0, k, ib))
    if not conjtrans:
        blocks = blocks[::-1]
    for i0 in blocks:
        sb = min(ib, k - i0)
        Vb = torch.tril(V[i0:m, i0:i0 + sb], -1)
        Vb[:sb, :sb] += torch.eye(sb, dtype=C.dtype)
        Tb = torch.triu(T[:sb, i0:i0 + sb])
        W = Vb.conj().T @ C[i0:]
        W = (Tb.conj().T if conjtrans else Tb) @ W
        C[i0:] -= Vb @ W


def _ref_tsqrt(A1, A2, T, ib, tri):
    m, n = A2.shape
    if tri:
        A2 *= torch.triu(torch.ones_like(A2, dtype=torch.bool)).to(A2.dtype)
    for i0 in range(0, n, ib):
        sb = min(ib, n - i0)
        taus = []
        for j in range(i0, i0 + sb):
            mj = min(m, j + 1) if tri else m
            beta, tau, scal = _larfg(A1[j, j].item(), A2[:mj, j])
            A2[:mj, j] *= scal
            A1[j, j] = beta
            taus.append(tau)
            for c in range(j + 1, i0 + sb):
                w = A1[j, c] + A2[:mj, j].conj() @ A2[:mj, c]
                f = _cj(tau) * w
                A1[j, c] -= f
                A2[:mj, c] -= A2[:mj, j] * f
        V2 = A2[:, i0:i0 + sb]
        Tb = torch.zeros(sb, sb, dtype=A2.dtype)
        for jj in range(sb):
            Tb[jj, jj] = taus[jj]
            if jj:
                y = V2[:, :jj].conj().T @ V2[:, jj]
                Tb[:jj, jj] = -taus[jj] * (Tb[:jj, :jj] @ y)
        T[:sb, i0:i0 + sb] = Tb
        if i0 + sb < n:
            W = A1[i0:i0 + sb, i0 + sb:] + V2.conj().T @ A2[:, i0 + sb:]
            W = Tb.conj().T @ W
            A1[i0:i0 + sb, i0 + sb:] -= W
            A2[:, i0 + sb:] -= V2 @ W


def _ref_tsmqr(A1, A2, V2, T, ib, k, conjtrans, tri):
    if tri:
        V2 = torch.triu(V2)
    blocks = list(range(0, k, ib))
    if not conjtrans:
        blocks = blocks[::-1]
    for i0 in blocks:
        sb = min(ib, k - i0)
        Vb = V2[:, i0:i0 + sb]
        Tb = torch.triu(T[:sb, i0:i0 + sb])
        W = A1[i0:i0 + sb] + Vb.conj().T @ A2
        W = (Tb.conj().T if conjtrans else Tb) @ W
        A1[i0:i0 + sb] -= W
        A2 -= Vb @ W


# ----------------------------------------------------------------------------- kinds
USE_MFMA_APPLY = True  # real precisions, m <= 256, ib <= 32: csrc/kernels/qr_mfma.hip


def view_flags(dtype: torch.dtype, transposed: bool):
    """(tr, cj) of a tile view: the tile itself, or its conjugate transpose."""
    return (1, 1 if dtype.is_complex else 0) if transposed else (0, 0)


@lru_cache(maxsize=None)
def kinds(dtype: torch.dtype, ib: int, av=(0, 0), vv=None):
    """The QR (or LQ, via transposed views) kind set for one precision / inner block size.

    Extents per task (m, n, k):
      geqrt  : tile rows, tile cols                         roles A(rw), T(rw)
      unmqr  : C rows, C cols, reflectors                   roles C(rw), V(r), T(r)
      tsqrt  : A2 rows, cols                                roles A1(rw), A2(rw), T(rw)
      tsmqr  : A2 rows, cols, reflectors                    roles A1(rw), A2(rw), V(r), T(r)
    ``*_h`` apply Q^H (conjtrans) else Q; ``tt*`` treat A2/V2 as upper triangular.
    ``av`` / ``vv``: (tr, cj) view flags of the A/C operands and of the
    reflector (V) operands (``view_flags``); vv defaults to av.  LQ = QR with
    av = vv = conjugate-transposed views; right-side application = transposed
    C view.  Extents are those of the (logical) transposed problem."""
    prec = _lib.prec_code(dtype)
    vv = av if vv is None else vv
    tr, cj = av
    vtr, vcj = vv
    out = {}
    pre = f"qr{tr}{cj}{vtr}{vcj}_"

    def mk(name, roles, exec_role, cfn, cname, flags, prio, fast=None, panel=None):
        """fast = (mode, conjtrans): eligible for the MFMA reflector-application kernel;
        panel = (ts, tri): eligible for the MFMA panel kernel."""
        def gpu(items_ptr, n, stream, emax):
            lib = _lib.load()
            if fast is not None and USE_MFMA_APPLY and lib.dpl_qr_apply_mfma_ok(prec, emax[0], ib):
                rc = lib.dpl_qr_apply_mfma(prec, n, items_ptr, emax[1], tr, vtr, ib, fast[1], fast[0], stream)
                _lib.check(rc, "qr_apply_mfma")
                return
            if panel is not None and USE_MFMA_APPLY and lib.dpl_qr_apply_mfma_ok(prec, emax[0], ib):
                rc = lib.dpl_qr_panel_mfma(prec, n, items_ptr, tr, ib, panel[0], panel[1], stream)
                _lib.check(rc, "qr_panel_mfma")
                return
            rc = getattr(lib, cname)(prec, n, items_ptr, *flags, stream)
            _lib.check(rc, cname)
        out[name] = Kind(pre + name + f"_{prec}_{ib}", roles, exec_role, gpu, cfn, prio=prio)

    # geqrt
    def c_geqrt(refs, ext):
        m, n, _ = ext
        A = _load(refs[0], m, n, tr, cj)
        Tt = torch.as_strided(refs[1][0], (ib, n), (1, refs[1][2]), refs[1][1])
        Tw = Tt.clone()
        _ref_geqrt(A, Tw, ib)
        _store(refs[0], A, tr, cj)
        Tt.copy_(Tw)
    mk("geqrt", (("A", RW, 1), ("T", RW, 3)), 0, c_geqrt, "dpl_geqrt", (tr, cj, ib), 0, panel=(0, 0))

    for conjtrans in (0, 1):
        def c_unmqr(refs, ext, conjtrans=conjtrans):
            m, n, k = ext
            C = _load(refs[0], m, n, tr, cj)
            V = _load(refs[1], m, k, vtr, vcj)
            Tt = torch.as_strided(refs[2][0], (ib, k), (1, refs[2][2]), refs[2][1])
            _ref_unmqr(C, V, Tt.clone(), ib, k, conjtrans)
            _store(refs[0], C, tr, cj)
        mk("unmqr" + ("_h" if conjtrans else ""), (("C", RW, 1), ("V", R, 2), ("T", R, 3)), 0, c_unmqr,
           "dpl_unmqr", (tr, cj, vtr, vcj, ib, conjtrans), 1, fast=(2, conjtrans))

    for tri in (0, 1):
        def c_tsqrt(refs, ext, tri=tri):
            m, n, _ = ext
            A1 = _load(refs[0], n, n, tr, cj)
            A2 = _load(refs[1], m, n, tr, cj)
            Tt = torch.as_strided(refs[2][0], (ib, n), (1, refs[2][2]), refs[2][1])
            Tw = Tt.clone()
            _ref_tsqrt(A1, A2, Tw, ib, tri)
            _store(refs[0], A1, tr, cj)
            # TT: the strictly lower part of A2 belongs to other reflectors -- never written
            _store(refs[1], A2, tr, cj, torch.triu(torch.ones(m, n, dtype=torch.bool)) if tri else None)
            Tt.copy_(Tw)
        mk(("tt" if tri else "ts") + "qrt", (("A1", RW, 0), ("A2", RW, 1), ("T", RW, 3)), 1, c_tsqrt,
           "dpl_tsqrt", (tr, cj, ib, tri), 0, panel=(1, tri))
        for conjtrans in (0, 1):
            def c_tsmqr(refs, ext, tri=tri, conjtrans=conjtrans):
                m, n, k = ext
                A1 = _load(refs[0], k, n, tr, cj)
                A2 = _load(refs[1], m, n, tr, cj)
                V2 = _load(refs[2], m, k, vtr, vcj)
                Tt = torch.as_strided(refs[3][0], (ib, k), (1, refs[3][2]), refs[3][1])
                _ref_tsmqr(A1, A2, V2, Tt.clone(), ib, k, conjtrans, tri)
                _store(refs[0], A1, tr, cj)
                _store(refs[1], A2, tr, cj)
            mk(("tt" if tri else "ts") + "mqr" + ("_h" if conjtrans else ""),
               (("A1", RW, 0), ("A2", RW, 1), ("V", R, 2), ("T", R, 3)), 1, c_tsmqr,
               "dpl_tsmqr", (tr, cj, vtr, vcj, ib, conjtrans, tri), 1, fast=(tri, conjtrans))
    return out

