"""Householder QR / LQ family on tile DAGs (flat TS trees).

Reference: ``src/zgeqrf.jdf`` (task classes zgeqrt(k) :98, zunmqr(k,n) :198,
ztsqrt(k,m) :314, ztsmqr(k,m,n) :443), ``src/zgelqf.jdf``, ``src/zunmqr_{LN,LC,
RN,RC}.jdf``, ``src/zunmlq_*.jdf``, ``src/zungqr.jdf``, ``src/zunglq.jdf`` and the
drivers ``src/zgeqrs_wrapper.c``, ``zgelqs_wrapper.c``, ``zgels_wrapper.c``.

Every algorithm here inserts tile tasks in program order into a
:class:`~dplasma_amd.runtime.dag.TileDAG`; the runtime levels the DAG and runs
each level as one batched launch per kernel kind (e.g. all the TSMQR updates
that are ready together -- typically thousands -- in one launch).

LQ is QR of A^H: the LQ algorithms run the QR task sequence on the *logical*
matrix X = A^H (tile (i, j) of X is A(j, i)^H) with kernels that read tiles
through conjugate-transposed views.  Right-side applications run the left-side
sequence on C^H.  T matrices keep the reference's layout (mt x nt tiles of
IB x NB, T(m, k) for the k-th panel's m-th kill in QR, T(k, n) in LQ).
"""
from __future__ import annotations

import numpy as np

from ..constants import (dplasmaConjTrans, dplasmaLeft, dplasmaLower, dplasmaNoTrans, dplasmaNonUnit, dplasmaRight,
                         dplasmaTrans, dplasmaUpper, dplasmaUpperLower)
from ..ops import qr_ops
from ..ops import tile_ops as ops
from ..ops.batch import TileBatch
from ..runtime.dag import TileDAG
from ..runtime.taskpool import Taskpool
from ..utils.flops import flops
from . import aux, blas3
from .cholesky import _Seq


class _L:
    """Logical tile view: M itself (t=False) or M^H (t=True)."""

    def __init__(self, M, t=False):
        self.M, self.t = M, t
        self.mt, self.nt = (M.nt, M.mt) if t else (M.mt, M.nt)
        self.m, self.n = (M.n, M.m) if t else (M.m, M.n)
        self._r = np.array([M.tile_cols(i) if t else M.tile_rows(i) for i in range(self.mt)], dtype=np.int64)
        self._c = np.array([M.tile_rows(j) if t else M.tile_cols(j) for j in range(self.nt)], dtype=np.int64)

    def rows(self, i):
        return self._r[i]

    def cols(self, j):
        return self._c[j]

    def keys(self, dag, i, j):
        i, j = np.broadcast_arrays(np.asarray(i, dtype=np.int64), np.asarray(j, dtype=np.int64))
        return dag.keys(self.M, j, i) if self.t else dag.keys(self.M, i, j)


def _ib_of(T):
    return T.mb


def _check_square_tiles(A):
    if A.mb != A.nb:
        raise ValueError("QR/LQ tile algorithms need square tiles (mb == nb)")


# ----------------------------------------------------------------------------- task sequences
def _factor(dag: TileDAG, X: _L, TT: _L, kd):
    """Flat-tree tile QR of the logical matrix X (zgeqrf.jdf task order)."""
    MT, NT = X.mt, X.nt
    for k in range(min(MT, NT)):
        rk, ck = int(X.rows(k)), int(X.cols(k))
        akk, tkk = X.keys(dag, k, k), TT.keys(dag, k, k)
        dag.add(kd["geqrt"], [[akk, tkk]], [[rk, ck, 0]])
        ns = np.arange(k + 1, NT)
        if len(ns):
            dag.add(kd["unmqr_h"], np.stack([X.keys(dag, k, ns), np.full(len(ns), akk), np.full(len(ns), tkk)], 1),
                    np.stack([np.full(len(ns), rk), X.cols(ns), np.full(len(ns), min(rk, ck))], 1))
        ms = np.arange(k + 1, MT)
        if not len(ms):
            continue
        dag.add(kd["tsqrt"], np.stack([np.full(len(ms), akk), X.keys(dag, ms, k), TT.keys(dag, ms, k)], 1),
                np.stack([X.rows(ms), np.full(len(ms), ck), np.zeros(len(ms), dtype=np.int64)], 1))
        if len(ns):
            mm, nn = np.meshgrid(ms, ns, indexing="ij")
            mm, nn = mm.ravel(), nn.ravel()
            dag.add(kd["tsmqr_h"], np.stack([X.keys(dag, k, nn), X.keys(dag, mm, nn), X.keys(dag, mm, k),
                                            TT.keys(dag, mm, k)], 1),
                    np.stack([X.rows(mm), X.cols(nn), np.full(len(mm), ck)], 1))


def _apply(dag: TileDAG, X: _L, TT: _L, C: _L, kd, conjtrans: bool, K: int = None):
    """C := Q^H C (conjtrans) or Q C, Q from _factor(X): the zunmqr_LC / zunmqr_LN sequences."""
    MT = X.mt
    K = min(X.mt, X.nt) if K is None else K
    NTc = C.nt
    ns = np.arange(NTc)
    ks = range(K) if conjtrans else range(K - 1, -1, -1)
    sfx = "_h" if conjtrans else ""
    for k in ks:
        rk, ck = int(X.rows(k)), int(X.cols(k))
        akk, tkk = X.keys(dag, k, k), TT.keys(dag, k, k)
        ms = np.arange(k + 1, MT)
        if not conjtrans:
            ms = ms[::-1]

        def unm():
            dag.add(kd["unmqr" + sfx],
                    np.stack([C.keys(dag, k, ns), np.full(NTc, akk), np.full(NTc, tkk)], 1),
                    np.stack([np.full(NTc, int(C.rows(k))), C.cols(ns), np.full(NTc, min(rk, ck))], 1))

        def tsm():
            if not len(ms):
                return
            mm, nn = np.meshgrid(ms, ns, indexing="ij")
            mm, nn = mm.ravel(), nn.ravel()
            dag.add(kd["tsmqr" + sfx], np.stack([C.keys(dag, k, nn), C.keys(dag, mm, nn), X.keys(dag, mm, k),
                                                TT.keys(dag, mm, k)], 1),
                    np.stack([C.rows(mm), C.cols(nn), np.full(len(mm), ck)], 1))
        if conjtrans:
            unm()
            tsm()
        else:
            tsm()
            unm()


def _kinds(A, T, logical_t, c_t=None):
    fa = qr_ops.view_flags(A.dtype, logical_t)
    fc = fa if c_t is None else qr_ops.view_flags(A.dtype, c_t)
    return qr_ops.kinds(A.dtype, _ib_of(T), fc, fa)


def _check_T(A, T):
    if T.mt < A.mt or T.nt < A.nt:
        raise ValueError("T must have as many tiles as A (mt x nt tiles of ib x nb)")
    if T.nb != A.nb or T.mb > 64:
        raise ValueError("T tiles must be ib x nb with ib <= 64")


# ----------------------------------------------------------------------------- GEQRF / GELQF
def geqrf_New(ctx, A, T) -> Taskpool:
    """Tile QR factorization A = Q R (dplasma_zgeqrf_New, src/zgeqrf_wrapper.c:130)."""
    _check_square_tiles(A)
    _check_T(A, T)
    dag = TileDAG(ctx, "geqrf")
    _factor(dag, _L(A), _L(T), _kinds(A, T, False))
    dag.flops = flops(A.prec, "geqrf", A.m, A.n)
    return dag.compile()


def geqrf(ctx, A, T):
    geqrf_New(ctx, A, T).execute(ctx)
    return 0


def gelqf_New(ctx, A, T) -> Taskpool:
    """Tile LQ factorization A = L Q (dplasma_zgelqf_New, src/zgelqf_wrapper.c:83)."""
    _check_square_tiles(A)
    _check_T(A, T)
    dag = TileDAG(ctx, "gelqf")
    _factor(dag, _L(A, True), _L(T, True), _kinds(A, T, True))
    dag.flops = flops(A.prec, "gelqf", A.m, A.n)
    return dag.compile()


def gelqf(ctx, A, T):
    gelqf_New(ctx, A, T).execute(ctx)
    return 0


# ----------------------------------------------------------------------------- UNMQR / UNMLQ
def _norm_trans(A, trans):
    if trans == dplasmaTrans:
        if A.dtype.is_complex:
            raise ValueError("trans=Trans is invalid for complex precisions (use ConjTrans)")
        return dplasmaConjTrans
    if trans not in (dplasmaNoTrans, dplasmaConjTrans):
        raise ValueError("invalid trans")
    return trans


def _unm(ctx, name, side, trans, A, T, C, lq: bool):
    _check_square_tiles(A)
    trans = _norm_trans(A, trans)
    if side not in (dplasmaLeft, dplasmaRight):
        raise ValueError("invalid side")
    # the effective left-side product on the logical C: see module docstring
    qh = trans == dplasmaConjTrans
    if lq:
        qh = not qh  # Q_A = Q_B^H
    c_t = side == dplasmaRight
    if c_t:
        qh = not qh  # C op(Q) = (op(Q)^H C^H)^H
    X = _L(A, lq)
    dag = TileDAG(ctx, name)
    K = min(A.mt, A.nt)
    _apply(dag, X, _L(T, lq), _L(C, c_t), _kinds(A, T, lq, c_t), qh, K)
    dag.flops = flops(A.prec, "unmqr", C.m, C.n, min(A.m, A.n), side == dplasmaLeft)
    return dag.compile()


def unmqr_New(ctx, side, trans, A, T, C) -> Taskpool:
    """C := op(Q) C or C op(Q), Q from geqrf (dplasma_zunmqr_New, src/zunmqr_wrapper.c:92)."""
    return _unm(ctx, "unmqr", side, trans, A, T, C, lq=False)


def unmqr(ctx, side, trans, A, T, C):
    unmqr_New(ctx, side, trans, A, T, C).execute(ctx)
    return 0


def unmlq_New(ctx, side, trans, A, T, C) -> Taskpool:
    """C := op(Q) C or C op(Q), Q from gelqf (dplasma_zunmlq_New, src/zunmlq_wrapper.c:91)."""
    return _unm(ctx, "unmlq", side, trans, A, T, C, lq=True)


def unmlq(ctx, side, trans, A, T, C):
    unmlq_New(ctx, side, trans, A, T, C).execute(ctx)
    return 0


# ----------------------------------------------------------------------------- UNGQR / UNGLQ
def _ung(ctx, name, A, T, Q, lq: bool):
    _check_square_tiles(A)
    init = aux.laset_New(ctx, dplasmaUpperLower, 0.0, 1.0, Q)
    dag = TileDAG(ctx, name)
    K = min(A.mt, A.nt)
    _apply(dag, _L(A, lq), _L(T, lq), _L(Q, lq), _kinds(A, T, lq, lq), False, K)
    if lq:
        dag.flops = flops(A.prec, "unglq", Q.m, Q.n, min(A.m, A.n))
    else:
        dag.flops = flops(A.prec, "ungqr", Q.m, Q.n, min(A.m, A.n))
    return _Seq(name, ctx, [init, dag.compile()])


def ungqr_New(ctx, A, T, Q) -> Taskpool:
    """Q := the first Q.n columns of the orthogonal factor of geqrf (src/zungqr_wrapper.c:73)."""
    return _ung(ctx, "ungqr", A, T, Q, lq=False)


def ungqr(ctx, A, T, Q):
    ungqr_New(ctx, A, T, Q).execute(ctx)
    return 0


def unglq_New(ctx, A, T, Q) -> Taskpool:
    """Q := the first Q.m rows of the orthogonal factor of gelqf (src/zunglq_wrapper.c:73)."""
    return _ung(ctx, "unglq", A, T, Q, lq=True)


def unglq(ctx, A, T, Q):
    unglq_New(ctx, A, T, Q).execute(ctx)
    return 0


# ----------------------------------------------------------------------------- solvers
def _zero_rows(ctx, B, r0):
    """B(r0:, :) := 0 (r0 need not be tile aligned)."""
    tb = TileBatch()
    for (m, n) in B.local_tiles():
        top = m * B.mb
        rows = B.tile_rows(m)
        if top + rows <= r0:
            continue
        skip = max(0, r0 - top)
        tb.add(B.offset(m, n) + skip, rows - skip, B.tile_cols(n))
    tb.finalize()
    if len(tb):
        ops.laset(0, 0.0, 0.0, B.data, B.ld, tb)
    if ctx.is_gpu:
        import torch
        torch.cuda.current_stream(ctx.device).synchronize()


def geqrs(ctx, A, T, B):
    """Least-squares solve after geqrf: B := Q^H B, B(0:N) := R^-1 B(0:N) (src/zgeqrs_wrapper.c)."""
    unmqr(ctx, dplasmaLeft, dplasmaConjTrans, A, T, B)
    N = A.n
    blas3.trsm(ctx, dplasmaLeft, dplasmaUpper, dplasmaNoTrans, dplasmaNonUnit, 1.0, A.submatrix(0, 0, N, N),
               B.submatrix(0, 0, N, B.n))
    return 0


def gelqs(ctx, A, T, B):
    """Minimum-norm solve after gelqf: B(0:M) := L^-1 B(0:M), B(M:N) := 0, B := Q^H B (src/zgelqs_wrapper.c)."""
    M = A.m
    blas3.trsm(ctx, dplasmaLeft, dplasmaLower, dplasmaNoTrans, dplasmaNonUnit, 1.0, A.submatrix(0, 0, M, M),
               B.submatrix(0, 0, M, B.n))
    if A.n > M:
        _zero_rows(ctx, B, M)
    unmlq(ctx, dplasmaLeft, dplasmaConjTrans, A, T, B)
    return 0


def gels(ctx, trans, A, T, B):
    """Least squares / minimum norm solutions of op(A) X = B (src/zgels_wrapper.c)."""
    trans = _norm_trans(A, trans)
    if B.m < max(A.m, A.n) and B.m < A.n:
        raise ValueError("B must have max(M, N) rows")
    M, N = A.m, A.n
    if M >= N:
        geqrf(ctx, A, T)
        if trans == dplasmaNoTrans:
            return geqrs(ctx, A, T, B)
        blas3.trsm(ctx, dplasmaLeft, dplasmaUpper, dplasmaConjTrans, dplasmaNonUnit, 1.0, A.submatrix(0, 0, N, N),
                   B.submatrix(0, 0, N, B.n))
        if M > N:
            _zero_rows(ctx, B, N)
        unmqr(ctx, dplasmaLeft, dplasmaNoTrans, A, T, B)
        return 0
    gelqf(ctx, A, T)
    if trans == dplasmaNoTrans:
        return gelqs(ctx, A, T, B)
    unmlq(ctx, dplasmaLeft, dplasmaNoTrans, A, T, B)
    blas3.trsm(ctx, dplasmaLeft, dplasmaLower, dplasmaConjTrans, dplasmaNonUnit, 1.0, A.submatrix(0, 0, M, M),
               B.submatrix(0, 0, M, B.n))
    return 0
