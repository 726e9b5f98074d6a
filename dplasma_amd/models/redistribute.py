"""Redistribution between descriptors (``parsec_redistribute`` analogue).

Used by transposed map operations on non-square grids and by the ScaLAPACK
compatibility layer (``src/scalapack_wrappers/common.c:27-128``) to move data
between a LAPACK-layout block-cyclic matrix and a tiled one.  One planned
all-to-all of whole tiles (``parallel.exchange``) followed by one batched copy
kernel on each rank.
"""
from __future__ import annotations

from ..constants import dplasmaNoTrans
from ..ops import tile_ops as ops
from ..ops.batch import TileBatch
from ..parallel.exchange import ExchangePlan


def transpose_into(ctx, A, trans):
    """Return a new descriptor T (A.n x A.m, same grid/tiling transposed) with T = op(A)."""
    from ..descriptor import TiledMatrix
    T = TiledMatrix(A.dtype, A.nb, A.mb, A.n, A.m, P=A.P, Q=A.Q, kp=A.grid.kp, kq=A.grid.kq, ip=A.grid.ip,
                    jq=A.grid.jq, rank=A.rank, device=A.device, storage=A.storage, name=A.name + "^T")
    needs = {}
    for r in range(ctx.world):
        pr, pc = r // T.Q, r % T.Q
        needs[r] = [(0, n, m) for n in range(T.nt) if T.grid.pcol(n) == pc
                    for m in range(T.mt) if T.grid.prow(m) == pr]
    plan = ExchangePlan(ctx, [A], needs, A.dtype, A.device)
    buf = plan.new_recv_buffer()
    plan.run(buf)
    tb = TileBatch()
    for (m, n) in T.local_tiles():
        tb.add(plan.offset(0, n, m), T.tile_rows(m), T.tile_cols(n), gi=m * T.mb, gj=n * T.nb, b_off=T.offset(m, n))
    tb.finalize()
    ops.geadd(0, trans, 1.0, buf, plan.ld, 0.0, T.data, T.ld, tb, copy=True)
    return T


def redistribute(ctx, src, dst, m=None, n=None, si=0, sj=0, di=0, dj=0):
    """dst[di:di+m, dj:dj+n] = src[si:si+m, sj:sj+n] for tile-aligned offsets and equal tile sizes."""
    m = src.m - si if m is None else m
    n = src.n - sj if n is None else n
    if src.mb != dst.mb or src.nb != dst.nb or si % src.mb or sj % src.nb or di % dst.mb or dj % dst.nb:
        return _redistribute_elementwise(ctx, src, dst, m, n, si, sj, di, dj)
    S = src.submatrix(si, sj, m, n)
    D = dst.submatrix(di, dj, m, n)
    needs = {}
    for r in range(ctx.world):
        pr, pc = r // D.Q, r % D.Q
        needs[r] = [(0, mm, nn) for nn in range(D.nt) if D.grid.pcol(nn + D.jt0) == pc
                    for mm in range(D.mt) if D.grid.prow(mm + D.it0) == pr]
    plan = ExchangePlan(ctx, [S], needs, S.dtype, D.device)
    buf = plan.new_recv_buffer()
    plan.run(buf)
    tb = TileBatch()
    for (mm, nn) in D.local_tiles():
        tb.add(plan.offset(0, mm, nn), D.tile_rows(mm), D.tile_cols(nn), b_off=D.offset(mm, nn))
    tb.finalize()
    ops.geadd(0, dplasmaNoTrans, 1.0, buf, plan.ld, 0.0, D.data, D.ld, tb, copy=True)
    return D


def _redistribute_elementwise(ctx, src, dst, m, n, si, sj, di, dj):
    """General (unaligned) redistribution through a dense all-gather -- small/compat use only."""
    import torch
    import torch.distributed as dist
    full = src.to_dense_local().to(src.device)
    if ctx.world > 1:
        dist.all_reduce(full)
    block = full[si:si + m, sj:sj + n]
    dense = dst.to_dense_local().to(dst.device)
    if ctx.world > 1:
        dist.all_reduce(dense)
    dense[di:di + m, dj:dj + n] = block
    dst.from_dense(dense)
    return dst
