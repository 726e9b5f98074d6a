"""Two-sided reductions to band form and the eigenvalue / singular value drivers.

Reference: ``src/zherbt_L.jdf`` / ``zherbt_U.jdf`` + ``src/zherbt_wrapper.c``
(Hermitian -> band, dplasma_zherbt_New(uplo, ib, A, T)), ``src/zhbrdt.jdf``
(band -> tridiagonal bulge chasing), ``src/zheev_wrapper.c:14-90`` (heev NoVec
= herbt -> diag_band_to_rect -> hbrdt -> dsterf), ``src/zgebrd_ge2gb.jdf`` +
``src/zgebrd_ge2gb_wrapper.c`` (general -> upper band bidiagonal, alternating
QR / LQ panel steps with hqr/svd trees, Band in LAPACK upper band storage
``AB(nb + i - j, j)``, ``:1144-1197``), ``tests/testing_zheev.c``,
``tests/testing_zhbrdt.c``, ``tests/testing_zgebrd_ge2gb.c``.

MI355X design
-------------
* **herbt / ge2gb** are one tile DAG each (runtime/dag.py): every panel step is
  a one-panel tile QR (GEQRT / TSQRT / TTQRT on the GPU panel kernels) whose
  reflectors are applied from the left by the batched MFMA apply kernels and --
  for the two-sided reductions -- from the right by the same kernels reading
  C through a conjugate-transposed tile view (no transposition pass).  Panel
  k+1 starts as soon as its column has been updated by step k (DAG levels),
  so panel and update work of successive steps overlap on the two streams.
  herbt keeps A Hermitian in full storage (both triangles are mirrored once
  up front), trading 2x flops in the trailing update for using the regular
  MFMA tile kernels instead of a separate symmetric-tile kernel family.
* **hbrdt** (band -> tridiagonal) is the native C++ Householder bulge chase
  (csrc/runtime/band.cpp): O(N^2 nb) latency-bound work on an (nb+1) x N band
  that is replicated on every rank (no communication); ``dsterf`` (LAPACK via
  scipy) gives the eigenvalues.
* Singular values of the ge2gb band come from the same chase applied to the
  Golub-Kahan matrix [[0, B], [B^H, 0]] under the perfect shuffle (a Hermitian
  band of width 2 nb - 1 whose eigenvalues are +-sigma).
"""
from __future__ import annotations

import numpy as np
import torch

from ..constants import (dplasmaConjTrans, dplasmaLower, dplasmaNoTrans, dplasmaNoVec, dplasmaTrans,
                         dplasmaUpper)
from ..descriptor import TiledMatrix
from ..ops import qr_ops
from ..parallel import comm
from ..runtime.dag import TileDAG
from ..runtime.tileprog import TileProgram
from ..utils.flops import flops
from . import qr, qrtree
from .cholesky import _Seq


def _ct(A):
    return dplasmaConjTrans if A.dtype.is_complex else dplasmaTrans


def _rt():
    from ..lib import _dplasma_rt
    return _dplasma_rt


def T_descriptor(A, ib: int) -> TiledMatrix:
    """Block-reflector storage for the reductions: mt x nt tiles of ib x nb (like geqrf's T)."""
    return TiledMatrix(A.dtype, ib, A.nb, A.mt * ib, A.nt * A.nb, P=A.grid.P, Q=A.grid.Q, rank=A.rank,
                       device=A.device, name="T")


# ----------------------------------------------------------------------------- Hermitian mirroring
def _mirror_New(ctx, A, uplo, band_only=False):
    """Copy the ``uplo`` triangle's conjugate transpose into the other one (tile-wise, any grid)."""
    prog = TileProgram(ctx, "mirror")
    ct = _ct(A)
    s = prog.stage("mirror")
    for n in range(A.nt):
        for m in range(n + 1, (min(A.mt, n + 2) if band_only else A.mt)):
            if uplo == dplasmaLower:
                s.copy((A, m, n), (A, n, m), trans=ct)
            else:
                s.copy((A, n, m), (A, m, n), trans=ct)
        s.copy((A, n, n), (A, n, n), part=4 if uplo == dplasmaLower else 3, trans=ct)
    return prog.compile()


# ----------------------------------------------------------------------------- HERBT
def herbt_New(ctx, uplo, ib, A, T, tree=None):
    """Reduce Hermitian A to band form (bandwidth nb) by two-sided tile QR (dplasma_zherbt_New).

    On exit the ``uplo`` band of A holds the band matrix (diagonal tiles and the
    triangular R factors of the sub-diagonal tiles); the reflectors stay in the
    lower sub-diagonal tiles with their block factors in T (mt x nt tiles of
    ib x nb).  ``tree``: elimination tree over the (mt-1) x nt sub-diagonal
    matrix (flat TS by default, as the reference)."""
    qr._check_square_tiles(A)
    if A.m != A.n:
        raise ValueError("herbt needs a square matrix")
    if uplo not in (dplasmaLower, dplasmaUpper):
        raise ValueError("illegal value of uplo")
    if T.mb != ib or T.nb != A.nb or T.mt < A.mt or T.nt < A.nt:
        raise ValueError("T must have mt x nt tiles of ib x nb")
    parts = [_mirror_New(ctx, A, uplo)]
    nb = A.nb
    if A.mt > 1:
        dag = TileDAG(ctx, "herbt")
        dag.flops = flops(A.prec, "herbt", A.n)
        kl = qr_ops.kinds(A.dtype, ib, (0, 0), (0, 0))
        kr = qr_ops.kinds(A.dtype, ib, qr_ops.view_flags(A.dtype, True), (0, 0))
        Xs = A.submatrix(nb, 0, A.m - nb, A.n)                     # panel k = rows k+1.. of column k
        X = qr._L(Xs)
        Tl = qr._L(T.submatrix(ib, 0, (A.mt - 1) * ib, A.n))
        C = qr._L(A.submatrix(nb, nb, A.m - nb, A.n - nb), True)   # logical row i = A column i+1
        tree = tree or qrtree.FlatTree(X.mt, X.nt)
        for k in range(min(X.mt, X.nt)):
            qr._factor(dag, X, Tl, Tl, kl, tree, ks=[k])                  # A(k+1:, k:) := Q^H A(k+1:, k:)
            qr._apply(dag, X, Tl, Tl, C, kr, True, tree, ks=[k], n0=k)   # A(k+1:, k+1:) := A(k+1:, k+1:) Q
        parts.append(dag.compile())
    if uplo == dplasmaUpper:
        parts.append(_mirror_New(ctx, A, dplasmaLower, band_only=True))
    return _Seq("herbt", ctx, parts)


def herbt(ctx, uplo, ib, A, T, tree=None):
    herbt_New(ctx, uplo, ib, A, T, tree).execute(ctx)
    return 0


# ----------------------------------------------------------------------------- band extraction
def _gather(ctx, ab: torch.Tensor) -> np.ndarray:
    if ctx.world > 1:
        comm.allreduce(ab)
    return ab.cpu().numpy()


def diag_band_to_rect(ctx, A, Band=None, uplo=dplasmaLower) -> np.ndarray:
    """The nb-band of A in LAPACK band storage, replicated on every rank
    (parsec diag_band_to_rect).  Lower: AB(i - j, j); Upper: AB(nb + i - j, j).
    If a ``Band`` descriptor ((nb+1) x N, one tile row) is given its local tiles are filled too."""
    nb, N = A.nb, min(A.m, A.n)
    ab = torch.zeros(nb + 1, N, dtype=A.dtype, device=A.device)
    d = torch.arange(nb + 1, device=A.device).view(-1, 1)
    for (m, n) in A.local_tiles():
        c0 = n * nb
        if c0 >= N:
            continue
        t = A.tile(m, n)
        rows, cols = t.shape
        cols = min(cols, N - c0)
        j = torch.arange(cols, device=A.device).view(1, -1)
        if m == n:
            i = j + d if uplo == dplasmaLower else j - (nb - d)     # band row d <-> tile row
            ok = (i >= 0) & (i < rows) & ((i >= j) if uplo == dplasmaLower else (i <= j))
        elif uplo == dplasmaLower and m == n + 1:
            i = j + d - nb                                           # upper triangle of A(k+1, k)
            ok = (i >= 0) & (i <= j) & (i < rows)
        elif uplo == dplasmaUpper and n == m + 1:
            i = j + d                                                # lower triangle of A(k, k+1)
            ok = (i < rows) & (d < nb)
        else:
            continue
        vals = t[i.clamp(0, rows - 1), j.expand_as(i)]
        ab[:, c0:c0 + cols] += torch.where(ok, vals, torch.zeros((), dtype=A.dtype, device=A.device))
    out = _gather(ctx, ab)
    if Band is not None:
        src = torch.from_numpy(out)
        for (m, n) in Band.local_tiles():
            t = Band.tile(m, n)
            c0 = n * Band.nb
            r = min(t.shape[0], nb + 1)
            t.zero_()
            t[:r].copy_(src[:r, c0:c0 + t.shape[1]].to(t.device))
    return out


# ----------------------------------------------------------------------------- HBRDT / HEEV
def hbrdt(ctx, band, b: int = None):
    """Hermitian band (LAPACK lower band storage, numpy/torch (ldab x N) or a Band
    descriptor) -> real symmetric tridiagonal (d, e) (dplasma_zhbrdt_New).
    Native C++ bulge chasing; runs redundantly on every rank."""
    if isinstance(band, TiledMatrix):
        band = _band_from_descriptor(ctx, band)
    if isinstance(band, torch.Tensor):
        band = band.cpu().numpy()
    band = np.asfortranarray(band)
    b = band.shape[0] - 1 if b is None else b
    return _rt().hbrdt(band, int(b))


def _band_from_descriptor(ctx, Band):
    ab = torch.zeros(Band.m, Band.n, dtype=Band.dtype, device=Band.device)
    for (m, n) in Band.local_tiles():
        t = Band.tile(m, n)
        ab[m * Band.mb:m * Band.mb + t.shape[0], n * Band.nb:n * Band.nb + t.shape[1]] = t
    return _gather(ctx, ab)


def sterf(d, e) -> np.ndarray:
    """Eigenvalues (ascending) of the symmetric tridiagonal (d, e) (LAPACK dsterf)."""
    from scipy.linalg import lapack
    d = np.asarray(d, dtype=np.float64)
    e = np.asarray(e, dtype=np.float64)
    if d.size == 0:
        return d
    w, info = lapack.dsterf(d.copy(), e.copy() if e.size else np.zeros(0))[:2]
    if info != 0:
        raise RuntimeError(f"dsterf failed to converge (info={info})")
    return w


def heev_New(ctx, jobz, uplo, A, W, Z=None, info=None, ib: int = None):
    """Eigenvalues of Hermitian A (dplasma_zheev_New; like the reference only jobz = NoVec).

    W: output eigenvalues (ascending), a length-N tensor or an N x 1 descriptor."""
    if jobz != dplasmaNoVec:
        raise NotImplementedError("heev: only jobz = dplasmaNoVec is implemented (as in the reference)")
    ib = ib or min(32, A.nb)
    T = T_descriptor(A, ib)
    red = herbt_New(ctx, uplo, ib, A, T)
    tp = _Seq("heev", ctx, [red])
    tp.flops = flops(A.prec, "heev", A.n)

    def _tail():
        ab = diag_band_to_rect(ctx, A, uplo=dplasmaLower)
        d, e = _rt().hbrdt(np.asfortranarray(ab), A.nb)
        w = sterf(d, e)
        _store_values(W, w)
        if info is not None:
            info[0] = 0
        return 0
    tp.on_complete(_tail)
    tp._T = T
    return tp


def _store_values(W, w: np.ndarray):
    wt = torch.from_numpy(np.ascontiguousarray(w))
    if isinstance(W, TiledMatrix):
        for (m, n) in W.local_tiles():
            t = W.tile(m, n)
            r0 = m * W.mb
            t[:, 0].copy_(wt[r0:r0 + t.shape[0]].to(W.dtype).to(t.device))
    elif W is not None:
        W[: len(w)] = wt.to(W.dtype).to(W.device)


def heev(ctx, jobz, uplo, A, W, Z=None, ib: int = None):
    heev_New(ctx, jobz, uplo, A, W, Z, ib=ib).execute(ctx)
    return 0


def eigvalsh(ctx, A, uplo=dplasmaLower, ib: int = None) -> np.ndarray:
    """Convenience: eigenvalues of Hermitian A (destroys A), as a numpy array."""
    w = torch.zeros(A.n, dtype=torch.float64)
    heev(ctx, dplasmaNoVec, uplo, A, w, ib=ib)
    return w.numpy()


# ----------------------------------------------------------------------------- GEBRD_GE2GB
def gebrd_ge2gbx_New(ctx, ib, qrtree_, lqtree_, A, TS, TT, TSl, TTl, Band=None):
    """General A (M >= N) -> upper band bidiagonal (bandwidth nb) by alternating
    QR (column k, rows k..) and LQ (row k, columns k+1..) tile panel steps
    (dplasma_zgebrd_ge2gbx_New without the R-bidiag pre-QR).

    qrtree_: QR tree over A (mt x nt); lqtree_: LQ tree over the logical matrix
    A(:, 1:)^H ((nt-1) x mt); TS/TT: QR block factors (mt x nt tiles of ib x nb),
    TSl/TTl: LQ block factors (same shape)."""
    qr._check_square_tiles(A)
    if A.m < A.n:
        raise NotImplementedError("ge2gb: M < N (reduce A^H instead)")
    nb = A.nb
    dag = TileDAG(ctx, "ge2gb")
    dag.flops = flops(A.prec, "gebrd", A.m, A.n)
    kq = qr_ops.kinds(A.dtype, ib, (0, 0), (0, 0))
    Xq = qr._L(A)
    TSq, TTq = qr._L(TS), qr._L(TT)
    if A.nt > 1:
        kl = qr_ops.kinds(A.dtype, ib, qr_ops.view_flags(A.dtype, True), qr_ops.view_flags(A.dtype, True))
        Xl = qr._L(A.submatrix(0, nb, A.m, A.n - nb), True)           # logical row i = A column i+1
        TSlv = qr._L(TSl.submatrix(0, nb, TSl.m, TSl.n - nb), True)
        TTlv = qr._L(TTl.submatrix(0, nb, TTl.m, TTl.n - nb), True)
    for k in range(A.nt):
        qr._factor(dag, Xq, TSq, TTq, kq, qrtree_, ks=[k])
        if k < A.nt - 1 and k < min(Xl.mt, Xl.nt):
            qr._factor(dag, Xl, TSlv, TTlv, kl, lqtree_, ks=[k])
    tp = dag.compile()
    tp.band = None

    def _done():
        tp.band = diag_band_to_rect(ctx, A, Band, uplo=dplasmaUpper)
        return 0
    tp.on_complete(_done)
    return tp


def gebrd_ge2gbx(ctx, ib, qrtree_, lqtree_, A, TS, TT, TSl, TTl, Band=None):
    tp = gebrd_ge2gbx_New(ctx, ib, qrtree_, lqtree_, A, TS, TT, TSl, TTl, Band)
    tp.execute(ctx)
    return tp.band


def gebrd_ge2gb_New(ctx, ib, A, Band=None):
    """dplasma_zgebrd_ge2gb_New: flat trees, internal block-factor storage."""
    TS, TT, TSl, TTl = (T_descriptor(A, ib) for _ in range(4))
    tp = gebrd_ge2gbx_New(ctx, ib, qrtree.FlatTree(A.mt, A.nt), qrtree.FlatTree(max(A.nt - 1, 1), A.mt),
                          A, TS, TT, TSl, TTl, Band)
    tp._T = (TS, TT, TSl, TTl)
    return tp


def gebrd_ge2gb(ctx, ib, A, Band=None):
    """Reduce A (M >= N) to upper band bidiagonal form; returns the band (LAPACK
    upper band storage, (nb+1) x N, replicated on every rank)."""
    tp = gebrd_ge2gb_New(ctx, ib, A, Band)
    tp.execute(ctx)
    return tp.band


def band_singular_values(ab: np.ndarray, kd: int = None) -> np.ndarray:
    """Singular values (descending) of the square upper band matrix in LAPACK
    upper band storage ab ((kd+1) x N): native bulge chase of the perfect-shuffled
    Golub-Kahan matrix, then dsterf."""
    ab = np.asarray(ab)
    kd = ab.shape[0] - 1 if kd is None else kd
    n = ab.shape[1]
    if n == 0:
        return np.zeros(0)
    # GK ordering: index 2j <-> column j of B, 2i+1 <-> row i of B; entries B(i, j), j >= i:
    #   j == i      : M(2i+1, 2i) = B(i, i)                 (offset 1)
    #   j > i       : M(2j, 2i+1) = conj(B(i, j))           (offset 2(j-i)-1)
    bw = max(2 * kd - 1, 1)
    gk = np.zeros((bw + 1, 2 * n), dtype=ab.dtype)
    for s in range(kd + 1):                      # s = j - i
        if s >= n:
            break
        diag = ab[kd - s, s:]                    # B(i, i+s), i = 0..n-s-1
        if s == 0:
            gk[1, 0:2 * n:2] = diag
        else:
            gk[2 * s - 1, 1:2 * (n - s):2] = np.conj(diag)
    d, e = _rt().hbrdt(np.asfortranarray(gk), bw)
    w = sterf(d, e)
    return np.maximum(w[::-1][:n], 0.0)            # eigenvalues are +-sigma: keep the top n


def gesvd_values(ctx, A, ib: int = None) -> np.ndarray:
    """Convenience: singular values of A (M >= N; destroys A) via ge2gb + band chase."""
    ib = ib or min(32, A.nb)
    ab = gebrd_ge2gb(ctx, ib, A)
    return band_singular_values(ab, A.nb)


# ----------------------------------------------------------------------------- HETRD (h2b + b2s)
def hetrd_h2b_New(ctx, uplo, ib, A, T):
    """Hermitian -> band (src/zhetrd_h2b_L.jdf): the herbt reduction."""
    return herbt_New(ctx, uplo, ib, A, T)


def hetrd_b2s(ctx, DE, b: int = None):
    """Band -> tridiagonal in place on a band descriptor DE ((nb+1) x N, LAPACK lower band
    storage; src/zhetrd_b2s.jdf): on exit row 0 holds d, row 1 holds e, the rest is zero.
    Returns (d, e)."""
    ab = _band_from_descriptor(ctx, DE)
    d, e = _rt().hbrdt(np.asfortranarray(ab), ab.shape[0] - 1 if b is None else int(b))
    out = np.zeros_like(ab)
    out[0, :len(d)] = d
    out[1, :len(e)] = e
    src = torch.from_numpy(out)
    for (m, n) in DE.local_tiles():
        t = DE.tile(m, n)
        r0, c0 = m * DE.mb, n * DE.nb
        t.copy_(src[r0:r0 + t.shape[0], c0:c0 + t.shape[1]].to(t.device))
    return d, e


def hetrd(ctx, uplo, ib, A, DE, T):
    """A = Q T Q^H with T real symmetric tridiagonal (dplasma_zhetrd, src/zhetrd_wrapper.c):
    h2b on A, band -> DE (diag_band_to_rect), b2s on DE.  Returns (d, e)."""
    herbt(ctx, uplo, ib, A, T)
    diag_band_to_rect(ctx, A, DE, uplo=dplasmaLower)
    return hetrd_b2s(ctx, DE, A.nb)
