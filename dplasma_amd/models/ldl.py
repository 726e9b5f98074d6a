"""LDL^H without pivoting, preceded by random butterfly transformations (RBT).

Reference: ``src/zhetrf.jdf`` (hetrf2_nopiv / hetrf_nopiv / trsm / hedrk /
gemdm / trmdm task classes, :54-336), ``src/ztrdsm.jdf`` (B := D^-1 B,
CORE_ztrdsm), ``src/ztrmdm.jdf`` (strict triangle times D^-1, CORE_ztrmdm),
``src/zhebut.jdf`` / ``zgebut.jdf`` / ``zgebmm.jdf`` + ``src/zhebut_wrapper.c``
(recursive butterfly U = B_0 B_1 ... B_{d-1}; each B_l is block diagonal with
2^l butterflies W = 1/sqrt(2) [R0 R1; R0 -R1], R diagonal with entries
exp((u - 0.5)/10)), ``tests/testing_zhebut.c`` (hebut + hetrf, then solve).

MI355X design: hetrf is a TileProgram (one batched launch per step and op
type, any P x Q grid): the diagonal tile's LDL^H comes from the no-pivot LU
panel kernel on a copy (U = D L^H), TRSM against L_kk^H, the rows of D are
divided out by the diagonal-scaling kernel (``k_diag_scale``) while a copy
W = L D feeds the MFMA GEMM update A(m,n) -= W(m,k) L(n,k)^H.  Butterflies are
applied as distributed products with per-tile generated butterfly matrices
(2 nonzeros per row) on P x Q grids; on one process each level is one element-wise
O(n^2) pass (``csrc/kernels/butterfly.hip``); ``N`` must be a multiple of 2^levels.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..constants import (dplasmaConjTrans, dplasmaLeft, dplasmaLower, dplasmaNoTrans, dplasmaRight, dplasmaTrans,
                         dplasmaUnit, dplasmaUpperLower)
from ..ops import tile_ops as ops
from ..ops.batch import MASK_LOWER, TileBatch
from ..parallel import comm
from ..runtime.tileprog import TileProgram
from ..utils import lcg
from ..utils.flops import flops
from . import blas3
from .gemm import gemm

N_ = dplasmaNoTrans


def _ct(A):
    return dplasmaConjTrans if A.dtype.is_complex else dplasmaTrans


def _ldl_tile(W, key, info, base):
    """No-pivot LU of the copy W(k,k): lower = L (unit), diag = D."""
    def fn(res):
        b, off, ld = res[key]
        n = W.tile_rows(key[1])
        ops.getrf_panel(b, off, n, W.tile_cols(key[2]), ld, None, info, base, pivot=False)
    return fn


def _scale(part, cols, kd, kb, rows, ncols, gi, gj):
    def fn(res):
        db, doff, dld = res[kd]
        bb, boff, bld = res[kb]
        tb = TileBatch().add(doff, rows, ncols, gi=gi, gj=gj, b_off=boff).finalize()
        ops.diag_scale(part, cols, db, dld, bb, bld, tb)
    return fn


# ----------------------------------------------------------------------------- HETRF (LDL^H, no pivoting)
def hetrf_New(ctx, A, info_out=None):
    """A = L D L^H (lower storage; L unit lower below the diagonal, D on the diagonal) (dplasma_zhetrf_New)."""
    if A.mb != A.nb:
        raise ValueError("hetrf needs square tiles")
    prog = TileProgram(ctx, "hetrf")
    prog.flops = flops(A.prec, "hetrf", A.n)
    info = torch.zeros(1, dtype=torch.int32, device=A.device)
    W = A.like(name="W")
    ct = _ct(A)
    mA, mW = prog.mid(A), prog.mid(W)
    for k in range(A.mt):
        # Hermitian copy of the diagonal tile (only its lower triangle is current)
        s = prog.stage(f"ldl({k})")
        s.copy((A, k, k), (W, k, k), part=dplasmaLower)
        s = prog.stage(f"ldl_sym({k})")
        s.copy((A, k, k), (W, k, k), part=4, trans=ct)   # strictly upper := lower^H
        s = prog.stage(f"ldl_tile({k})")
        s.batch_fn([(W, k, k)], [], _ldl_tile(W, (mW, k, k), info, k * A.mb))
        s = prog.stage(f"ldl_back({k})")
        s.copy((W, k, k), (A, k, k), part=dplasmaLower)
        if k + 1 >= A.mt:
            continue
        s = prog.stage(f"trsm({k})")
        for m in range(k + 1, A.mt):
            s.trsm(dplasmaRight, dplasmaLower, ct, dplasmaUnit, 1.0, (A, k, k), (A, m, k))   # -> L(m,k) D_k
        s = prog.stage(f"keepW({k})")
        for m in range(k + 1, A.mt):
            s.copy((A, m, k), (W, m, k))
        s = prog.stage(f"scale({k})")
        for m in range(k + 1, A.mt):
            s.batch_fn([(A, m, k)], [(A, k, k)],
                       _scale(0, True, (mA, k, k), (mA, m, k), A.tile_rows(m), A.tile_cols(k), m * A.mb, k * A.nb))
        s = prog.stage(f"update({k})")
        for m in range(k + 1, A.mt):
            for n in range(k + 1, m + 1):
                s.gemm((A, m, n), [((W, m, k), N_, (A, n, k), ct)], alpha=-1.0, beta=1.0,
                       mask=MASK_LOWER if m == n else 0)
    tp = prog.compile()
    tp.info = info
    tp._W = W

    def _done():
        v = info.clone()
        comm.allreduce(v, op=torch.distributed.ReduceOp.MAX)
        r = int(v.item())
        if info_out is not None:
            info_out[0] = r
        return r
    tp.on_complete(_done)
    return tp


def hetrf(ctx, A):
    return hetrf_New(ctx, A).execute(ctx)


# ----------------------------------------------------------------------------- TRDSM / TRMDM
def trdsm_New(ctx, A, B):
    """B := D^-1 B with D the diagonal of A (dplasma_ztrdsm_New)."""
    prog = TileProgram(ctx, "trdsm")
    mA, mB = prog.mid(A), prog.mid(B)
    s = prog.stage("trdsm")
    for k in range(B.mt):
        for n in range(B.nt):
            s.batch_fn([(B, k, n)], [(A, k, k)],
                       _scale(0, False, (mA, k, k), (mB, k, n), B.tile_rows(k), B.tile_cols(n), k * B.mb, n * B.nb))
    return prog.compile()


def trdsm(ctx, A, B):
    trdsm_New(ctx, A, B).execute(ctx)
    return 0


def trmdm_New(ctx, A):
    """Strictly lower part of A := L D^-1 column-wise (dplasma_ztrmdm_New / CORE_ztrmdm lower)."""
    prog = TileProgram(ctx, "trmdm")
    mA = prog.mid(A)
    s = prog.stage("trmdm")
    for k in range(A.nt):
        for m in range(k, A.mt):
            s.batch_fn([(A, m, k)], [(A, k, k)],
                       _scale(3 if m == k else 0, True, (mA, k, k), (mA, m, k), A.tile_rows(m), A.tile_cols(k),
                              m * A.mb, k * A.nb))
    return prog.compile()


def trmdm(ctx, A):
    trmdm_New(ctx, A).execute(ctx)
    return 0


def hetrs(ctx, A, B, U_but=None):
    """Solve with the hetrf factors (and the butterfly of hebut, if given): x = U (L D L^H)^-1 U^T b."""
    if U_but is not None:
        gebmm(ctx, B, U_but, _ct(B))
    blas3.trsm(ctx, dplasmaLeft, dplasmaLower, N_, dplasmaUnit, 1.0, A, B)
    trdsm(ctx, A, B)
    blas3.trsm(ctx, dplasmaLeft, dplasmaLower, _ct(A), dplasmaUnit, 1.0, A, B)
    if U_but is not None:
        gebmm(ctx, B, U_but, N_)
    return 0


# ----------------------------------------------------------------------------- butterflies
def butterfly_vectors(n: int, levels: int, seed: int = 3872) -> torch.Tensor:
    """levels x n random diagonals, entries exp((u - 0.5) / 10), u uniform in [0, 1) (RBT_zrandom)."""
    u = lcg.rnd_block(0, 0, n * levels, 1, n * levels, seed, False)[:, 0] + 0.5
    return torch.from_numpy(np.exp((u - 0.5) / 10.0)).reshape(levels, n)


def _butterfly_descriptor(like, n, level, r, transpose=False):
    """The n x n butterfly matrix B_level (2^level diagonal blocks of size n / 2^level) on like's grid."""
    from ..descriptor import TiledMatrix
    Bm = TiledMatrix(like.dtype, like.mb, like.mb, n, n, P=like.grid.P, Q=like.grid.Q, rank=like.rank,
                     device=like.device, name=f"B{level}")
    size = n >> level
    h = size // 2
    s2 = 1.0 / math.sqrt(2.0)
    for (m, c) in Bm.local_tiles():
        r0, c0 = m * Bm.mb, c * Bm.nb
        rows, cols = Bm.tile_rows(m), Bm.tile_cols(c)
        I = torch.arange(r0, r0 + rows).view(-1, 1).expand(rows, cols)
        J = torch.arange(c0, c0 + cols).view(1, -1).expand(rows, cols)
        if transpose:
            I, J = J, I
        blk_i, blk_j = I // size, J // size
        li, lj = I % size, J % size
        same = blk_i == blk_j
        top = li < h
        p = torch.where(top, li, li - h)                  # partner index within the half
        base = blk_i * size
        v = torch.zeros(rows, cols, dtype=torch.float64)
        r0v = r[(base + p).clamp(max=n - 1)]
        r1v = r[(base + h + p).clamp(max=n - 1)]
        v = torch.where(same & (lj == p), r0v * s2, v)
        v = torch.where(same & (lj == h + p), torch.where(top, r1v * s2, -r1v * s2), v)
        Bm.tile(m, c).copy_(v.to(like.dtype).to(like.device))
    if like.device.type == "cuda":
        torch.cuda.synchronize(like.device)
    return Bm


def _elementwise(A) -> bool:
    """One process: each level is one element-wise pass (O(n^2), ops.butterfly -- the reference's HEBUT /
    GEBUT / GEBMM segment updates, src/cores/core_zhebut.c:21-46).  On a P x Q grid the row / column
    partners of a level live on other ranks; there the level is a distributed product with the
    generated butterfly matrix (2 nonzeros per row)."""
    return A.grid.P * A.grid.Q == 1


def gebmm(ctx, A, U_but, trans=N_):
    """A := U A (trans = NoTrans) or U^T A (Trans/ConjTrans), U = B_0 B_1 ... B_{d-1} from U_but (dplasma_zgebmm)."""
    levels, n = U_but.shape
    if A.m != n:
        raise ValueError("butterfly order does not match A")
    order = range(levels - 1, -1, -1) if trans == N_ else range(levels)
    if _elementwise(A):
        for l in order:
            ops.butterfly(A, U_but[l], n >> l, dplasmaLeft, trans)
        return 0
    for l in order:
        Bm = _butterfly_descriptor(A, n, l, U_but[l], transpose=(trans != N_))
        T = A.like(name="T")
        gemm(ctx, N_, N_, 1.0, Bm, A, 0.0, T)
        A.data.copy_(T.data)
    return 0


def gebut(ctx, A, U_but, V_but=None):
    """A := U^T A V for general A (dplasma_zgebut); V defaults to U."""
    V_but = U_but if V_but is None else V_but
    gebmm(ctx, A, U_but, dplasmaTrans)
    levels, n = V_but.shape
    if _elementwise(A):
        for l in range(levels):
            ops.butterfly(A, V_but[l], n >> l, dplasmaRight, N_)
        return 0
    for l in range(levels):
        Bm = _butterfly_descriptor(A, n, l, V_but[l])
        T = A.like(name="T")
        gemm(ctx, N_, N_, 1.0, A, Bm, 0.0, T)
        A.data.copy_(T.data)
    return 0


def hebut(ctx, A, levels: int = 2, seed: int = 3872):
    """A := U^H A U with a random recursive butterfly of depth ``levels`` (dplasma_zhebut);
    returns U_but (levels x N), needed by hetrs to map solutions back.  A must be
    stored full (both triangles); on exit both triangles hold U^H A U."""
    n = A.n
    if A.m != A.n or n % (1 << levels):
        raise ValueError("hebut needs a square matrix whose order is a multiple of 2^levels")
    U = butterfly_vectors(n, levels, seed)
    gebut(ctx, A, U, U)
    return U
