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
from ..runtime import capped
from ..runtime.dag import TileDAG
from ..runtime.taskpool import Taskpool
from ..utils.flops import flops
from . import aux, blas3, qr_panel, qrtree
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
def _runs(kills):
    """Split a panel's kill list into maximal runs of one kernel class (TS / TT)."""
    out = []
    for (p, m, t) in kills:
        cls = "ts" if t == qrtree.KILLED_BY_TS else "tt"
        if out and out[-1][0] == cls:
            out[-1][1].append(p)
            out[-1][2].append(m)
        else:
            out.append((cls, [p], [m]))
    return [(c, np.array(p, dtype=np.int64), np.array(m, dtype=np.int64)) for c, p, m in out]


def _factor(dag: TileDAG, X: _L, TS: _L, TT: _L, kd, tree, ks=None):
    """Tile QR of the logical matrix X along the elimination plan of ``tree``
    (only the panels in ``ks`` if given: one-sided panel steps of the
    two-sided band reductions in models/eigen.py).

    Per panel k (zgeqrf.jdf / zgeqrf_param.jdf task classes): GEQRT on every
    head row, UNMQR of the head rows' trailing tiles, then the kills in plan
    order (TSQRT/TTQRT on the panel, TSMQR/TTMQR on the trailing tiles)."""
    MT, NT = X.mt, X.nt
    for k in (range(min(MT, NT)) if ks is None else ks):
        ck = int(X.cols(k))
        heads = np.array(tree.heads(k), dtype=np.int64)
        ns = np.arange(k + 1, NT)
        dag.add(kd["geqrt"], np.stack([X.keys(dag, heads, k), TS.keys(dag, heads, k)], 1),
                np.stack([X.rows(heads), np.full(len(heads), ck), np.zeros(len(heads), dtype=np.int64)], 1))
        if len(ns):
            hh, nn = (x.ravel() for x in np.meshgrid(heads, ns, indexing="ij"))
            dag.add(kd["unmqr_h"], np.stack([X.keys(dag, hh, nn), X.keys(dag, hh, k), TS.keys(dag, hh, k)], 1),
                    np.stack([X.rows(hh), X.cols(nn), np.minimum(X.rows(hh), ck)], 1))
        for cls, pv, vm in _runs(tree.kills(k)):
            Tm = TS if cls == "ts" else TT
            dag.add(kd[cls + "qrt"], np.stack([X.keys(dag, pv, k), X.keys(dag, vm, k), Tm.keys(dag, vm, k)], 1),
                    np.stack([X.rows(vm), np.full(len(vm), ck), np.zeros(len(vm), dtype=np.int64)], 1))
            if len(ns):
                ii, nn = (x.ravel() for x in np.meshgrid(np.arange(len(vm)), ns, indexing="ij"))
                dag.add(kd[cls + "mqr_h"], np.stack([X.keys(dag, pv[ii], nn), X.keys(dag, vm[ii], nn),
                                                    X.keys(dag, vm[ii], k), Tm.keys(dag, vm[ii], k)], 1),
                        np.stack([X.rows(vm[ii]), X.cols(nn), np.full(len(ii), ck)], 1))


def _factor_rec(dag: TileDAG, X: _L, TS: _L, TT: _L, kd, tree, hnb: int):
    """_factor with the reference's RECURSIVE task bodies (src/zgeqrf.jdf:126,220,347,509, under
    dplasma_zgeqrf_setrecursive): every tile task on tiles wider than ``hnb`` runs as sub-tasks on
    hnb-wide column blocks of its tiles (zgeqrfr_geqrt / zgeqrfr_tsqrt / zgeqrfr_unmqr / zgeqrfr_tsmqr):

      GEQRT(k)        block j: GEQRT of rows j.. x block j (T columns of block j), UNMQR of rows j..
                      x the blocks right of it, with block j's reflectors;
      TSQRT(m, k)     block j: TSQRT of the triangle (j, j) of the head tile over block j of the killed
                      tile, TSMQR of the head rows j.. / killed tile columns right of block j;
      UNMQR / TSMQR   independent updates of the hnb-wide column blocks of the updated tiles.

    With hnb a multiple of IB (the T tile height) every sub-task computes exactly the reflectors and
    T blocks of the whole-tile kernel.  TT kills (triangle on triangle) stay whole-tile tasks."""
    MT, NT = X.mt, X.nt
    z = np.zeros(2, dtype=np.int64)

    def blocks(w):
        return [(c, min(hnb, w - c)) for c in range(0, w, hnb)]

    for k in range(min(MT, NT)):
        ck = int(X.cols(k))
        heads = [int(h) for h in tree.heads(k)]
        ns = list(range(k + 1, NT))
        for h in heads:
            rk = int(X.rows(h))
            for j0, w in blocks(min(ck, rk)):
                dag.add(kd["geqrt"], [[X.keys(dag, h, k), TS.keys(dag, h, k)]], [[rk - j0, w, 0]],
                        sub=[[[j0, j0], [0, j0]]])
                if j0 + w < ck:
                    dag.add(kd["unmqr_h"], [[X.keys(dag, h, k), X.keys(dag, h, k), TS.keys(dag, h, k)]],
                            [[rk - j0, ck - j0 - w, min(rk - j0, w)]], sub=[[[j0, j0 + w], [j0, j0], [0, j0]]])
            for n in ns:
                cn = int(X.cols(n))
                for c0, w in blocks(cn):
                    dag.add(kd["unmqr_h"], [[X.keys(dag, h, n), X.keys(dag, h, k), TS.keys(dag, h, k)]],
                            [[rk, w, min(rk, ck)]], sub=[[[0, c0], z, z]])
        for cls, pv, vm in _runs(tree.kills(k)):
            Tm = TS if cls == "ts" else TT
            for p_, m_ in zip(pv.tolist(), vm.tolist()):
                rm = int(X.rows(m_))
                if cls == "ts":
                    for j0, w in blocks(ck):
                        dag.add(kd["tsqrt"], [[X.keys(dag, p_, k), X.keys(dag, m_, k), Tm.keys(dag, m_, k)]],
                                [[rm, w, 0]], sub=[[[j0, j0], [0, j0], [0, j0]]])
                        if j0 + w < ck:
                            dag.add(kd["tsmqr_h"], [[X.keys(dag, p_, k), X.keys(dag, m_, k), X.keys(dag, m_, k),
                                                     Tm.keys(dag, m_, k)]],
                                    [[rm, ck - j0 - w, w]], sub=[[[j0, j0 + w], [0, j0 + w], [0, j0], [0, j0]]])
                else:
                    dag.add(kd["ttqrt"], [[X.keys(dag, p_, k), X.keys(dag, m_, k), Tm.keys(dag, m_, k)]],
                            [[rm, ck, 0]])
                for n in ns:
                    cn = int(X.cols(n))
                    for c0, w in blocks(cn):
                        dag.add(kd[cls + "mqr_h"], [[X.keys(dag, p_, n), X.keys(dag, m_, n), X.keys(dag, m_, k),
                                                     Tm.keys(dag, m_, k)]],
                                [[rm, w, ck]], sub=[[[0, c0], [0, c0], z, z]])


def _apply(dag: TileDAG, X: _L, TS: _L, TT: _L, C: _L, kd, conjtrans: bool, tree, K: int = None, ks=None,
           n0: int = 0):
    """C := Q^H C (conjtrans) or Q C, Q from _factor(X, tree) (zunmqr_L{C,N}[_param].jdf).
    ``ks``: apply only these panels' reflectors; ``n0``: only C's columns n0.. ."""
    K = min(X.mt, X.nt) if K is None else K
    NTc = C.nt
    ns = np.arange(n0, NTc)
    sfx = "_h" if conjtrans else ""
    if ks is None:
        ks = range(K) if conjtrans else range(K - 1, -1, -1)
    for k in ks:
        ck = int(X.cols(k))
        heads = np.array(tree.heads(k), dtype=np.int64)

        def unm():
            hh, nn = (x.ravel() for x in np.meshgrid(heads, ns, indexing="ij"))
            dag.add(kd["unmqr" + sfx], np.stack([C.keys(dag, hh, nn), X.keys(dag, hh, k), TS.keys(dag, hh, k)], 1),
                    np.stack([C.rows(hh), C.cols(nn), np.minimum(X.rows(hh), ck)], 1))

        runs = _runs(tree.kills(k))
        if not conjtrans:
            runs = [(c, p[::-1], m[::-1]) for (c, p, m) in runs[::-1]]
        else:
            unm()
        for cls, pv, vm in runs:
            Tm = TS if cls == "ts" else TT
            ii, nn = (x.ravel() for x in np.meshgrid(np.arange(len(vm)), ns, indexing="ij"))
            dag.add(kd[cls + "mqr" + sfx], np.stack([C.keys(dag, pv[ii], nn), C.keys(dag, vm[ii], nn),
                                                    X.keys(dag, vm[ii], k), Tm.keys(dag, vm[ii], k)], 1),
                    np.stack([C.rows(vm[ii]), C.cols(nn), np.full(len(ii), ck)], 1))
        if not conjtrans:
            unm()


def _panel_format(A, T, tree):
    """The apply must use the stacked-domain engine: it can handle A and T was written by it (the tile
    engines -- PTG-style DAG or DTD -- mark their per-tile TSQRT layout with qr_format = "tile")."""
    return qr_panel.usable(A, tree) and getattr(T, "qr_format", "panel") == "panel"


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
    flat = qrtree.FlatTree(A.mt, A.nt)
    if qr_panel.usable(A, flat) and not capped.wanted(ctx, [A, T]):
        tp = qr_panel.factor_New(ctx, A, T, T, flat, "geqrf")
    else:
        T.full_T = {}   # tile engine: the panel engine's kept T factors no longer describe T
        T.qr_format = "tile"
        dag = TileDAG(ctx, "geqrf")
        _factor(dag, _L(A), _L(T), _L(T), _kinds(A, T, False), qrtree.FlatTree(A.mt, A.nt))
        dag.flops = flops(A.prec, "geqrf", A.m, A.n)
        tp = dag.compile()
    tp._rec_build = lambda hnb: _recursive_New(ctx, "geqrf", A, T, T, flat, hnb)
    return tp


def _recursive_New(ctx, name, A, TS, TT, tree, hnb):
    """The tile-engine factorisation with recursive (hnb-wide column block) task bodies -- what
    dplasma_zgeqrf_setrecursive turns a geqrf taskpool into (see _factor_rec)."""
    ib = TS.mb
    hnb = max(ib, (int(hnb) // ib) * ib)
    TS.full_T, TT.full_T = {}, {}
    TS.qr_format = TT.qr_format = "tile"
    dag = TileDAG(ctx, name + "_rec")
    _factor_rec(dag, _L(A), _L(TS), _L(TT), _kinds(A, TS, False), tree, hnb)
    dag.flops = flops(A.prec, "geqrf", A.m, A.n)
    tp = dag.compile()
    tp.recursive_nb = hnb
    return tp


def geqrf(ctx, A, T):
    geqrf_New(ctx, A, T).execute(ctx)
    return 0


def gelqf_New(ctx, A, T) -> Taskpool:
    """Tile LQ factorization A = L Q (dplasma_zgelqf_New, src/zgelqf_wrapper.c:83)."""
    _check_square_tiles(A)
    _check_T(A, T)
    dag = TileDAG(ctx, "gelqf")
    _factor(dag, _L(A, True), _L(T, True), _L(T, True), _kinds(A, T, True), qrtree.FlatTree(A.nt, A.mt))
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


def _flat(A, lq):
    return qrtree.FlatTree(A.nt, A.mt) if lq else qrtree.FlatTree(A.mt, A.nt)


def _unm(ctx, name, side, trans, A, T, C, lq: bool, tree=None, TT=None):
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
    if not lq and _panel_format(A, T, tree or _flat(A, lq)):
        return qr_panel.apply_New(ctx, side, trans, A, T, TT if TT is not None else T, C, tree or _flat(A, lq), name)
    X = _L(A, lq)
    dag = TileDAG(ctx, name)
    K = min(A.mt, A.nt)
    _apply(dag, X, _L(T, lq), _L(TT if TT is not None else T, lq), _L(C, c_t), _kinds(A, T, lq, c_t), qh,
           tree or _flat(A, lq), K)
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
def _ung(ctx, name, A, T, Q, lq: bool, tree=None, TT=None):
    _check_square_tiles(A)
    init = aux.laset_New(ctx, dplasmaUpperLower, 0.0, 1.0, Q)
    if not lq and _panel_format(A, T, tree or _flat(A, lq)):
        app = qr_panel.apply_New(ctx, dplasmaLeft, dplasmaNoTrans, A, T, TT if TT is not None else T, Q,
                                 tree or _flat(A, lq), name)
        app.flops = flops(A.prec, "ungqr", Q.m, Q.n, min(A.m, A.n))
        return _Seq(name, ctx, [init, app])
    dag = TileDAG(ctx, name)
    K = min(A.mt, A.nt)
    _apply(dag, _L(A, lq), _L(T, lq), _L(TT if TT is not None else T, lq), _L(Q, lq), _kinds(A, T, lq, lq), False,
           tree or _flat(A, lq), K)
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


# ----------------------------------------------------------------------------- hierarchical (tree-parameterised) variants
def _check_tree(A, tree, lq):
    mt, nt = (A.nt, A.mt) if lq else (A.mt, A.nt)
    if tree.mt != mt or tree.nt != nt:
        raise ValueError(f"qrtree built for {tree.mt}x{tree.nt} tiles, matrix has {mt}x{nt}")


def geqrf_param_New(ctx, tree, A, TS, TT) -> Taskpool:
    """Hierarchical QR driven by a reduction tree (dplasma_zgeqrf_param_New, src/zgeqrf_param_wrapper.c).

    TS receives the T factors of GEQRT/TSQRT, TT those of TTQRT."""
    _check_square_tiles(A)
    _check_T(A, TS)
    _check_T(A, TT)
    _check_tree(A, tree, False)
    if qr_panel.usable(A, tree) and not capped.wanted(ctx, [A, TS, TT]):
        tp = qr_panel.factor_New(ctx, A, TS, TT, tree, "geqrf_param")
    else:
        TS.full_T, TT.full_T = {}, {}   # tile engine: drop the panel engine's kept T factors
        TS.qr_format = TT.qr_format = "tile"
        dag = TileDAG(ctx, "geqrf_param")
        _factor(dag, _L(A), _L(TS), _L(TT), _kinds(A, TS, False), tree)
        dag.flops = flops(A.prec, "geqrf", A.m, A.n)
        tp = dag.compile()
    tp._rec_build = lambda hnb: _recursive_New(ctx, "geqrf_param", A, TS, TT, tree, hnb)
    return tp


def geqrf_param(ctx, tree, A, TS, TT):
    geqrf_param_New(ctx, tree, A, TS, TT).execute(ctx)
    return 0


def gelqf_param_New(ctx, tree, A, TS, TT) -> Taskpool:
    """Hierarchical LQ (dplasma_zgelqf_param_New); ``tree`` built with trans=ConjTrans."""
    _check_square_tiles(A)
    _check_T(A, TS)
    _check_T(A, TT)
    _check_tree(A, tree, True)
    dag = TileDAG(ctx, "gelqf_param")
    _factor(dag, _L(A, True), _L(TS, True), _L(TT, True), _kinds(A, TS, True), tree)
    dag.flops = flops(A.prec, "gelqf", A.m, A.n)
    return dag.compile()


def gelqf_param(ctx, tree, A, TS, TT):
    gelqf_param_New(ctx, tree, A, TS, TT).execute(ctx)
    return 0


def unmqr_param_New(ctx, side, trans, tree, A, TS, TT, C) -> Taskpool:
    _check_tree(A, tree, False)
    return _unm(ctx, "unmqr_param", side, trans, A, TS, C, lq=False, tree=tree, TT=TT)


def unmqr_param(ctx, side, trans, tree, A, TS, TT, C):
    unmqr_param_New(ctx, side, trans, tree, A, TS, TT, C).execute(ctx)
    return 0


def unmlq_param_New(ctx, side, trans, tree, A, TS, TT, C) -> Taskpool:
    _check_tree(A, tree, True)
    return _unm(ctx, "unmlq_param", side, trans, A, TS, C, lq=True, tree=tree, TT=TT)


def unmlq_param(ctx, side, trans, tree, A, TS, TT, C):
    unmlq_param_New(ctx, side, trans, tree, A, TS, TT, C).execute(ctx)
    return 0


def ungqr_param_New(ctx, tree, A, TS, TT, Q) -> Taskpool:
    _check_tree(A, tree, False)
    return _ung(ctx, "ungqr_param", A, TS, Q, lq=False, tree=tree, TT=TT)


def ungqr_param(ctx, tree, A, TS, TT, Q):
    ungqr_param_New(ctx, tree, A, TS, TT, Q).execute(ctx)
    return 0


def unglq_param_New(ctx, tree, A, TS, TT, Q) -> Taskpool:
    _check_tree(A, tree, True)
    return _ung(ctx, "unglq_param", A, TS, Q, lq=True, tree=tree, TT=TT)


def unglq_param(ctx, tree, A, TS, TT, Q):
    unglq_param_New(ctx, tree, A, TS, TT, Q).execute(ctx)
    return 0


def geqrs_param(ctx, tree, A, TS, TT, B):
    """Least squares after geqrf_param (dplasma_zgeqrs_param)."""
    unmqr_param(ctx, dplasmaLeft, dplasmaConjTrans, tree, A, TS, TT, B)
    N = A.n
    blas3.trsm(ctx, dplasmaLeft, dplasmaUpper, dplasmaNoTrans, dplasmaNonUnit, 1.0, A.submatrix(0, 0, N, N),
               B.submatrix(0, 0, N, B.n))
    return 0


def gelqs_param(ctx, tree, A, TS, TT, B):
    """Minimum-norm solve after gelqf_param (dplasma_zgelqs_param)."""
    M = A.m
    blas3.trsm(ctx, dplasmaLeft, dplasmaLower, dplasmaNoTrans, dplasmaNonUnit, 1.0, A.submatrix(0, 0, M, M),
               B.submatrix(0, 0, M, B.n))
    if A.n > M:
        _zero_rows(ctx, B, M)
    unmlq_param(ctx, dplasmaLeft, dplasmaConjTrans, tree, A, TS, TT, B)
    return 0
