"""Auxiliary distributed operations: generators, map operations, norms.

Reference roles:
* generators  -- ``dplasma_zplrnt/zplghe/zplgsy`` (``src/zplrnt_wrapper.c:111``,
  ``src/zplghe_wrapper.c:95``, ``src/zplgsy_wrapper.c:97``) built on
  ``parsec_apply_New`` over local tiles;
* map ops     -- ``dplasma_zlaset/zlacpy/zgeadd/ztradd/zlascal``
  (``src/zlaset_wrapper.c:93``, ``src/zlacpy_wrapper.c:90``,
  ``src/zgeadd_wrapper.c:119``, ``src/zlascal_wrapper.c:112``, ``src/map2.jdf``);
* norms       -- ``dplasma_zlange/zlanhe/zlansy/zlantr``
  (``src/zlange_wrapper.c:75`` ..., ``src/zlange_frb_cyclic.jdf``): per-tile
  partials, reduction over the process grid, result broadcast to every rank.

Each operation is one batched kernel launch over all local tiles (GPU) plus,
for norms, one small all-reduce.
"""
from __future__ import annotations

import math

import torch

from ..constants import (dplasmaConjTrans, dplasmaFrobeniusNorm, dplasmaInfNorm, dplasmaLower, dplasmaMaxNorm,
                         dplasmaNoTrans, dplasmaOneNorm, dplasmaTrans, dplasmaUnit, dplasmaUpper, dplasmaUpperLower)
from ..ops import tile_ops as ops
from ..ops.batch import TileBatch
from ..parallel import comm
from ..runtime import Taskpool


def local_tile_batch(A, uplo=dplasmaUpperLower, B=None, transB=False) -> TileBatch:
    """TileBatch of A's local tiles (tile-level triangle selection); b_off from B's same tile."""
    tb = TileBatch()
    for (m, n) in A.local_tiles(uplo):
        b_off = 0
        if B is not None:
            b_off = B.offset(n, m) if transB else B.offset(m, n)
        tb.add(A.offset(m, n), A.tile_rows(m), A.tile_cols(n), gi=m * A.mb, gj=n * A.nb, b_off=b_off)
    return tb.finalize()


def _single(ctx, name, fn) -> Taskpool:
    tp = Taskpool(name, ctx)
    tp.task(name, "update", fn)
    return tp.finish_build()


# ----------------------------------------------------------------------------- generators
def plrnt_New(ctx, A, seed: int) -> Taskpool:
    tb = local_tile_batch(A)
    return _single(ctx, "plrnt", lambda: ops.generate("rnt", A.data, A.ld, tb, A.m, seed))


def plghe_New(ctx, bump: float, uplo: int, A, seed: int) -> Taskpool:
    tb = local_tile_batch(A, uplo)
    return _single(ctx, "plghe", lambda: ops.generate("ghe", A.data, A.ld, tb, A.m, seed, bump))


def plgsy_New(ctx, bump, uplo: int, A, seed: int) -> Taskpool:
    tb = local_tile_batch(A, uplo)
    return _single(ctx, "plgsy", lambda: ops.generate("gsy", A.data, A.ld, tb, A.m, seed, bump))


def plrnt(ctx, *args):
    """plrnt(ctx, A, seed) or the reference form plrnt(ctx, diagdom, A, seed) (src/zplrnt_wrapper.c:191).

    diagdom: add max(M,N) (real) / (M+N-1) + i max(M,N) (complex) to the
    diagonal, making the matrix diagonally dominant (zplrnt_wrapper.c:45-60)."""
    if len(args) == 3:
        diagdom, A, seed = args
    else:
        (A, seed), diagdom = args, 0
    plrnt_New(ctx, A, seed).execute(ctx)
    if diagdom:
        mx = max(A.m, A.n)
        alpha = complex(A.m + A.n - 1, mx) if A.dtype.is_complex else float(mx)
        for (m, n) in A.local_tiles():
            if m + A.it0 == n + A.jt0:
                A.tile(m, n).diagonal().add_(alpha)
    return 0


def plghe(ctx, bump, uplo, A, seed):
    return plghe_New(ctx, bump, uplo, A, seed).execute(ctx)


def plgsy(ctx, bump, uplo, A, seed):
    return plgsy_New(ctx, bump, uplo, A, seed).execute(ctx)


# ----------------------------------------------------------------------------- map operations
def laset_New(ctx, uplo, alpha, beta, A) -> Taskpool:
    tb = local_tile_batch(A, uplo)
    return _single(ctx, "laset", lambda: ops.laset(uplo, alpha, beta, A.data, A.ld, tb))


def laset(ctx, uplo, alpha, beta, A):
    return laset_New(ctx, uplo, alpha, beta, A).execute(ctx)


def lacpy_New(ctx, uplo, A, B) -> Taskpool:
    """B := A on the uplo part (A and B share the distribution)."""
    tb = local_tile_batch(A, uplo, B=B)
    return _single(ctx, "lacpy", lambda: ops.geadd(uplo, dplasmaNoTrans, 1.0, A.data, A.ld, 0.0, B.data, B.ld, tb,
                                                   copy=True))


def lacpy(ctx, uplo, A, B):
    return lacpy_New(ctx, uplo, A, B).execute(ctx)


def geadd_New(ctx, trans, alpha, A, beta, B, uplo=dplasmaUpperLower) -> Taskpool:
    """B := alpha op(A) + beta B.  With trans, A's tile (n, m) must be local where B's (m, n) is
    (true for square grids); otherwise the operation is routed through a transposed redistribution."""
    if trans != dplasmaNoTrans and ctx.world > 1:
        from .redistribute import transpose_into
        At = transpose_into(ctx, A, trans)
        return geadd_New(ctx, dplasmaNoTrans, alpha, At, beta, B, uplo)
    tb = TileBatch()
    for (m, n) in B.local_tiles(uplo):
        a_off = A.offset(n, m) if trans != dplasmaNoTrans else A.offset(m, n)
        tb.add(a_off, B.tile_rows(m), B.tile_cols(n), gi=m * B.mb, gj=n * B.nb, b_off=B.offset(m, n))
    tb.finalize()
    # geadd kernel: item a_off -> source, b_off -> destination
    return _single(ctx, "geadd", lambda: ops.geadd(uplo, trans, alpha, A.data, A.ld, beta, B.data, B.ld, tb))


def geadd(ctx, trans, alpha, A, beta, B):
    return geadd_New(ctx, trans, alpha, A, beta, B).execute(ctx)


def tradd(ctx, uplo, trans, alpha, A, beta, B):
    return geadd_New(ctx, trans, alpha, A, beta, B, uplo=uplo).execute(ctx)


def lascal_New(ctx, uplo, alpha, A) -> Taskpool:
    tb = local_tile_batch(A, uplo)
    return _single(ctx, "lascal", lambda: ops.lascal(uplo, alpha, A.data, A.ld, tb))


def lascal(ctx, uplo, alpha, A):
    return lascal_New(ctx, uplo, alpha, A).execute(ctx)


# ----------------------------------------------------------------------------- norms
_PF, _PL, _PU, _PSL, _PSU, _PD = 0, 1, 2, 3, 4, 5


def _tiles(A, tile_uplo):
    return list(A.local_tiles(tile_uplo))


def _norm_parts(ctx, A, kind, part, unit, tiles):
    tb = TileBatch()
    for (m, n) in tiles:
        tb.add(A.offset(m, n), A.tile_rows(m), A.tile_cols(n), gi=m * A.mb, gj=n * A.nb)
    tb.finalize()
    return ops.tile_norm(kind, part, unit, A.data, A.ld, tb), tiles


def _reduce(t: torch.Tensor, op):
    comm.allreduce(t, op=op)
    return t


def _combine(ctx, A, norm, pieces):
    """pieces: list of (kind, partials, tiles, use_rows_as_cols) -> scalar norm (identical on all ranks)."""
    dev = A.device
    if norm == dplasmaMaxNorm:
        v = torch.zeros(1, dtype=torch.float64, device=dev)
        for kind, part, tiles, _ in pieces:
            if part.numel():
                v = torch.maximum(v, part.max().view(1))
        _reduce(v, torch.distributed.ReduceOp.MAX)
        return float(v.item())
    if norm == dplasmaFrobeniusNorm:
        scales = torch.zeros(1, dtype=torch.float64, device=dev)
        for kind, part, tiles, w in pieces:
            if part.numel():
                scales = torch.maximum(scales, part[:, 0].max().view(1))
        _reduce(scales, torch.distributed.ReduceOp.MAX)
        s = scales.item()
        tot = torch.zeros(1, dtype=torch.float64, device=dev)
        if s > 0:
            for kind, part, tiles, w in pieces:
                if part.numel():
                    tot += w * (part[:, 1] * (part[:, 0] / s) ** 2).sum()
        _reduce(tot, torch.distributed.ReduceOp.SUM)
        return float(s * math.sqrt(max(tot.item(), 0.0)))
    # one / inf: accumulate per global column (or row) sums
    length = A.n if norm == dplasmaOneNorm else A.m
    acc = torch.zeros(length + 1, dtype=torch.float64, device=dev)
    for kind, part, tiles, mirror in pieces:
        if not len(tiles) or not part.numel():
            continue
        # kind COLSUM indexes tile columns (n), ROWSUM tile rows (m): one scatter-add for every tile (was a
        # slice add per tile -- 16384 launches for a 64k matrix of 512-tiles)
        if kind == ops.NORM_COLSUM:
            bc = [(n * A.nb, A.tile_cols(n)) for (_, n) in tiles]
        else:
            bc = [(m * A.mb, A.tile_rows(m)) for (m, _) in tiles]
        bc = torch.tensor(bc, dtype=torch.int64)
        w = part.shape[1]
        col = torch.arange(w, dtype=torch.int64)
        valid = col[None, :] < bc[:, 1:2]
        idx = (bc[:, 0:1] + col[None, :])[valid]
        acc.index_add_(0, idx.to(dev), part[:len(tiles)][valid.to(part.device)].to(acc.dtype))
    _reduce(acc, torch.distributed.ReduceOp.SUM)
    return float(acc.max().item()) if length > 0 else 0.0


def lange(ctx, norm, A) -> float:
    """General matrix norm (max / one / inf / Frobenius)."""
    tiles = _tiles(A, dplasmaUpperLower)
    if norm == dplasmaMaxNorm:
        p, _ = _norm_parts(ctx, A, ops.NORM_MAX, _PF, False, tiles)
        return _combine(ctx, A, norm, [(ops.NORM_MAX, p, tiles, 1.0)])
    if norm == dplasmaFrobeniusNorm:
        p, _ = _norm_parts(ctx, A, ops.NORM_SSQ, _PF, False, tiles)
        return _combine(ctx, A, norm, [(ops.NORM_SSQ, p, tiles, 1.0)])
    kind = ops.NORM_COLSUM if norm == dplasmaOneNorm else ops.NORM_ROWSUM
    p, _ = _norm_parts(ctx, A, kind, _PF, False, tiles)
    return _combine(ctx, A, norm, [(kind, p, tiles, False)])


def lantr(ctx, norm, uplo, diag, A) -> float:
    """Norm of the uplo-trapezoid of A (unit diagonal if diag == Unit)."""
    tiles = _tiles(A, uplo)
    part = _PL if uplo == dplasmaLower else _PU
    unit = diag == dplasmaUnit
    if norm == dplasmaMaxNorm:
        p, _ = _norm_parts(ctx, A, ops.NORM_MAX, part, unit, tiles)
        return _combine(ctx, A, norm, [(ops.NORM_MAX, p, tiles, 1.0)])
    if norm == dplasmaFrobeniusNorm:
        p, _ = _norm_parts(ctx, A, ops.NORM_SSQ, part, unit, tiles)
        return _combine(ctx, A, norm, [(ops.NORM_SSQ, p, tiles, 1.0)])
    kind = ops.NORM_COLSUM if norm == dplasmaOneNorm else ops.NORM_ROWSUM
    p, _ = _norm_parts(ctx, A, kind, part, unit, tiles)
    return _combine(ctx, A, norm, [(kind, p, tiles, False)])


def lansy(ctx, norm, uplo, A, hermitian=False) -> float:
    """Norm of a symmetric/Hermitian matrix stored in its uplo triangle."""
    tiles = _tiles(A, uplo)
    tri = _PL if uplo == dplasmaLower else _PU
    strict = _PSL if uplo == dplasmaLower else _PSU
    if norm == dplasmaMaxNorm:
        p, _ = _norm_parts(ctx, A, ops.NORM_MAX, tri, False, tiles)
        return _combine(ctx, A, norm, [(ops.NORM_MAX, p, tiles, 1.0)])
    if norm == dplasmaFrobeniusNorm:
        ps, _ = _norm_parts(ctx, A, ops.NORM_SSQ, strict, False, tiles)
        pd, _ = _norm_parts(ctx, A, ops.NORM_SSQ, _PD, False, tiles)
        return _combine(ctx, A, norm, [(ops.NORM_SSQ, ps, tiles, 2.0), (ops.NORM_SSQ, pd, tiles, 1.0)])
    # one == inf for symmetric: column sums of the triangle + mirrored row sums of the strict part
    if uplo == dplasmaLower:
        pc, _ = _norm_parts(ctx, A, ops.NORM_COLSUM, tri, False, tiles)
        pr, _ = _norm_parts(ctx, A, ops.NORM_ROWSUM, strict, False, tiles)
        # row sums of lower tile (m, n) contribute to columns of block m
        return _combine(ctx, A, dplasmaOneNorm, [(ops.NORM_COLSUM, pc, tiles, False),
                                                 (ops.NORM_ROWSUM, pr, tiles, True)])
    pr, _ = _norm_parts(ctx, A, ops.NORM_ROWSUM, tri, False, tiles)
    pc, _ = _norm_parts(ctx, A, ops.NORM_COLSUM, strict, False, tiles)
    return _combine(ctx, A, dplasmaInfNorm, [(ops.NORM_ROWSUM, pr, tiles, False),
                                             (ops.NORM_COLSUM, pc, tiles, True)])


def lanhe(ctx, norm, uplo, A) -> float:
    return lansy(ctx, norm, uplo, A, hermitian=True)


# ----------------------------------------------------------------------------- apply / map2 (user tile operators)
def apply(ctx, uplo, A, op, op_args=None):
    """Run ``op(tile, uplo, m, n, op_args)`` on every local tile of the uplo part (parsec_apply_New).

    ``tile`` is a (rows x cols) column-major view of the tile's storage on the
    tile's device; the operator may modify it in place."""
    for (m, n) in A.local_tiles(uplo if uplo in (dplasmaLower, dplasmaUpper) else dplasmaUpperLower):
        t_uplo = uplo if m == n else dplasmaUpperLower
        op(A.tile(m, n), t_uplo, m, n, op_args)
    return 0


def map2(ctx, uplo, trans, A, B, op, op_args=None):
    """``op(tileA, tileB, uplo, m, n, op_args)`` on every local tile pair (dplasma_map2, src/map2.jdf).

    trans != NoTrans pairs B(m, n) with op(A)(m, n) = A(n, m)^T/^H: A is first
    redistributed transposed onto B's distribution."""
    if trans != dplasmaNoTrans:
        from .redistribute import transpose_into
        A = transpose_into(ctx, A, trans)
    for (m, n) in B.local_tiles(uplo if uplo in (dplasmaLower, dplasmaUpper) else dplasmaUpperLower):
        t_uplo = uplo if m == n else dplasmaUpperLower
        op(A.tile(m, n), B.tile(m, n), t_uplo, m, n, op_args)
    return 0


# ----------------------------------------------------------------------------- 2-norm estimate
def lanm2(ctx, A, info=None, tol=1e-10, maxiter=500) -> float:
    """Estimate ||A||_2 by power iteration on A^H A (dplasma_zlanm2, src/zlanm2.jdf:53-653).

    Every product is a distributed tile GEMM; returns the estimate and, if
    ``info`` (a list) is given, stores the iteration count (negative if the
    iteration did not converge)."""
    from .gemm import gemm_New
    X = A.__class__(A.dtype, A.nb, 1, A.n, 1, P=A.grid.P, Q=A.grid.Q, rank=A.rank, device=A.device, name="x")
    Y = A.__class__(A.dtype, A.mb, 1, A.m, 1, P=A.grid.P, Q=A.grid.Q, rank=A.rank, device=A.device, name="y")
    ct = dplasmaConjTrans if A.dtype.is_complex else dplasmaTrans
    laset(ctx, dplasmaUpperLower, 1.0 / math.sqrt(max(A.n, 1)), 1.0 / math.sqrt(max(A.n, 1)), X)
    # the two products are compiled once and re-executed every iteration
    ax = gemm_New(ctx, dplasmaNoTrans, dplasmaNoTrans, 1.0, A, X, 0.0, Y)
    ahy = gemm_New(ctx, ct, dplasmaNoTrans, 1.0, A, Y, 0.0, X)
    e, e0, it = 0.0, -1.0, 0
    while it < maxiter and abs(e - e0) > tol * max(e, 1e-300):
        e0 = e
        ax.execute(ctx)
        ahy.execute(ctx)
        nx = lange(ctx, dplasmaFrobeniusNorm, X)
        ny = lange(ctx, dplasmaFrobeniusNorm, Y)
        if nx == 0.0 or ny == 0.0:
            e = 0.0
            break
        e = nx / ny
        lascal(ctx, dplasmaUpperLower, 1.0 / nx, X)
        it += 1
    if info is not None:
        info.append(it if abs(e - e0) <= tol * max(e, 1e-300) else -it)
    return e


# ----------------------------------------------------------------------------- print
def print_matrix(ctx, uplo, A, file=None) -> int:
    """Print the uplo part of A tile by tile (dplasma_zprint, src/zprint.jdf PRINT_F/L/U).

    Local tiles are collected on rank 0 and printed in (m, n) order."""
    import sys
    out = file or sys.stdout
    dense = A.to_dense_local()
    if ctx.world > 1:
        import torch.distributed as dist
        parts = [None] * ctx.world
        dist.all_gather_object(parts, dense)
        dense = sum(parts)
    if ctx.rank != 0:
        return 0
    for n in range(A.nt):
        for m in range(A.mt):
            if (uplo == dplasmaLower and m < n) or (uplo == dplasmaUpper and m > n):
                continue
            r0, c0 = m * A.mb, n * A.nb
            t = dense[r0:r0 + A.tile_rows(m), c0:c0 + A.tile_cols(n)]
            print(f"{A.name}({m},{n}) [{t.shape[0]}x{t.shape[1]}]", file=out)
            for i in range(t.shape[0]):
                print("  " + " ".join(f"{complex(v):.6g}" if t.is_complex() else f"{float(v): .6e}" for v in t[i]),
                      file=out)
    return 0
