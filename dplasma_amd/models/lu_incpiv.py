"""LU factorization with incremental (tile-pairwise) pivoting.

Reference: ``src/zgetrf_incpiv.jdf`` (zgetrf(k) :52, zgessm(k,n) :102,
ztstrf(k,m) :156, zssssm(k,m,n) :234), ``src/ztrsmpl_incpiv.jdf`` and the
wrappers ``src/zgetrf_incpiv_wrapper.c:86``, ``src/ztrsmpl_incpiv_wrapper.c:75``,
``zgesv_incpiv``.  Descriptor shapes follow ``tests/testing_zgetrf_incpiv.c:51-62``:
L is (MT*IB) x N with IB x NB tiles, IPIV is M x NT integers with MB x 1 tiles.

The algorithm is a program-order tile DAG (runtime/dag.py): each step's
TSTRF chain and the SSSSM updates it releases become batched launches.
Pivoting is local to tile pairs, so unlike partial pivoting the panel needs no
cross-process reduction -- every grid shape is supported.
"""
from __future__ import annotations

import numpy as np
import torch

from ..constants import dplasmaLeft, dplasmaNoTrans, dplasmaNonUnit, dplasmaUpper
from ..descriptor import TiledMatrix
from ..ops import lu_incpiv_ops
from ..runtime.dag import TileDAG
from ..runtime.taskpool import Taskpool
from ..utils.flops import flops
from . import blas3


def L_descriptor(ctx, A, ib, name="L") -> TiledMatrix:
    """(MT*IB) x N matrix of IB x NB tiles, distributed like A."""
    return TiledMatrix(A.dtype, ib, A.nb, A.mt * ib, A.n, P=A.grid.P, Q=A.grid.Q, kp=A.grid.kp, kq=A.grid.kq,
                       ip=A.grid.ip, jq=A.grid.jq, rank=A.rank, device=A.device, name=name)


def ipiv_descriptor(ctx, A, name="IPIV") -> TiledMatrix:
    """M x NT integer matrix of MB x 1 tiles, distributed like A."""
    return TiledMatrix(torch.int32, A.mb, 1, A.m, A.nt, P=A.grid.P, Q=A.grid.Q, kp=A.grid.kp, kq=A.grid.kq,
                       ip=A.grid.ip, jq=A.grid.jq, rank=A.rank, device=A.device, name=name)


def _info(ctx):
    return torch.zeros(1, dtype=torch.int32, device=ctx.device)


def _extents(A):
    r = np.array([A.tile_rows(i) for i in range(A.mt)], dtype=np.int64)
    c = np.array([A.tile_cols(j) for j in range(A.nt)], dtype=np.int64)
    return r, c


def getrf_incpiv_New(ctx, A, L, IPIV, info_out=None) -> Taskpool:
    """A = P L U by tiles with incremental pivoting (dplasma_zgetrf_incpiv_New)."""
    if A.mb != A.nb:
        raise ValueError("getrf_incpiv needs square tiles")
    ib = L.mb
    if ib > 32:
        raise ValueError("IB must be <= 32")
    info = info_out if info_out is not None else _info(ctx)
    kd = lu_incpiv_ops.kinds(A.dtype, ib, A.nb, info)
    dag = TileDAG(ctx, "getrf_incpiv")
    rows, cols = _extents(A)
    K = lambda M, m, n: dag.keys(M, m, n)  # noqa: E731
    for k in range(min(A.mt, A.nt)):
        akk, pkk = K(A, k, k), K(IPIV, k, k)
        dag.add(kd["getrf"], [[akk, pkk]], [[rows[k], cols[k], k * A.nb]])
        ns = np.arange(k + 1, A.nt)
        if len(ns):
            dag.add(kd["gessm"], np.stack([K(A, k, ns), np.full(len(ns), akk), np.full(len(ns), pkk)], 1),
                    np.stack([np.full(len(ns), rows[k]), cols[ns], np.full(len(ns), min(rows[k], cols[k]))], 1))
        for m in range(k + 1, A.mt):
            dag.add(kd["tstrf"], [[akk, K(A, m, k), K(L, m, k), K(IPIV, m, k)]], [[rows[m], cols[k], k * A.nb]])
            if len(ns):
                dag.add(kd["ssssm"], np.stack([K(A, k, ns), K(A, m, ns), np.full(len(ns), K(L, m, k)),
                                               np.full(len(ns), K(IPIV, m, k)), np.full(len(ns), K(A, m, k))], 1),
                        np.stack([np.full(len(ns), rows[m]), cols[ns], np.full(len(ns), cols[k])], 1))
    dag.flops = flops(A.prec, "getrf", A.m, A.n)
    tp = dag.compile()
    tp.info = info

    def _done():
        v = info.clone()
        if ctx.world > 1:
            import torch.distributed as dist
            vv = v.to(ctx.device)
            dist.all_reduce(vv, op=dist.ReduceOp.MAX)
            v = vv
        return int(v.item())
    tp.on_complete(_done)
    return tp


def getrf_incpiv(ctx, A, L, IPIV):
    return getrf_incpiv_New(ctx, A, L, IPIV).execute(ctx)


def trsmpl_incpiv_New(ctx, A, L, IPIV, B) -> Taskpool:
    """B := L^-1 P B with the factors of getrf_incpiv (dplasma_ztrsmpl_incpiv_New)."""
    ib = L.mb
    info = _info(ctx)
    kd = lu_incpiv_ops.kinds(A.dtype, ib, A.nb, info)
    dag = TileDAG(ctx, "trsmpl_incpiv")
    rows, cols = _extents(A)
    brows = np.array([B.tile_rows(i) for i in range(B.mt)], dtype=np.int64)
    bcols = np.array([B.tile_cols(j) for j in range(B.nt)], dtype=np.int64)
    K = lambda M, m, n: dag.keys(M, m, n)  # noqa: E731
    ns = np.arange(B.nt)
    for k in range(min(A.mt, A.nt)):
        akk, pkk = K(A, k, k), K(IPIV, k, k)
        dag.add(kd["gessm"], np.stack([K(B, k, ns), np.full(len(ns), akk), np.full(len(ns), pkk)], 1),
                np.stack([np.full(len(ns), brows[k]), bcols, np.full(len(ns), min(rows[k], cols[k]))], 1))
        for m in range(k + 1, A.mt):
            dag.add(kd["ssssm"], np.stack([K(B, k, ns), K(B, m, ns), np.full(len(ns), K(L, m, k)),
                                           np.full(len(ns), K(IPIV, m, k)), np.full(len(ns), K(A, m, k))], 1),
                    np.stack([np.full(len(ns), brows[m]), bcols, np.full(len(ns), cols[k])], 1))
    dag.flops = flops(A.prec, "trsm", True, A.n, B.n)
    return dag.compile()


def trsmpl_incpiv(ctx, A, L, IPIV, B):
    trsmpl_incpiv_New(ctx, A, L, IPIV, B).execute(ctx)
    return 0


def gesv_incpiv(ctx, A, L, IPIV, B):
    """Solve A X = B with incremental-pivoting LU (dplasma_zgesv_incpiv)."""
    info = getrf_incpiv(ctx, A, L, IPIV)
    if info != 0:
        return info
    trsmpl_incpiv(ctx, A, L, IPIV, B)
    blas3.trsm(ctx, dplasmaLeft, dplasmaUpper, dplasmaNoTrans, dplasmaNonUnit, 1.0, A, B)
    return 0
