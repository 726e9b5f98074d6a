"""Level-3 BLAS on distributed tiled matrices.

Reference wrappers: ``src/ztrsm_wrapper.c:95`` (8 JDF variants ztrsm_{LLN..RUT}),
``src/ztrmm_wrapper.c:96`` (8 variants), ``src/zherk_wrapper.c:81``,
``src/zsyrk_wrapper.c:81``, ``src/zher2k_wrapper.c:87``, ``src/zsyr2k_wrapper.c:87``,
``src/zhemm_wrapper.c:86``, ``src/zsymm_wrapper.c:88``, ``src/zger_wrapper.c:48``.

All variants are expressed as owner-computes TileProgram stages whose heavy
work is the batched MFMA GEMM engine (and the batched TRSM kernel for the
diagonal solves); there is one code path per operation instead of eight JDF
files: op(A) is resolved to "which stored tile, which transpose" and the
substitution order (forward/backward) from the effective triangle.
"""
from __future__ import annotations

from ..constants import (dplasmaConjTrans, dplasmaLeft, dplasmaLower, dplasmaNoTrans, dplasmaNonUnit, dplasmaRight,
                         dplasmaTrans, dplasmaUnit, dplasmaUpper, dplasmaUpperLower)
from ..ops.batch import MASK_LOWER, MASK_UPPER
from ..runtime.tileprog import TileProgram
from ..utils.flops import flops

N_, T_, C_ = dplasmaNoTrans, dplasmaTrans, dplasmaConjTrans
P_LOWER, P_UPPER, P_SLOWER, P_SUPPER, P_DIAG = 1, 2, 3, 4, 5


def _op_tile(A, trans, i, j):
    """op(A) tile (i, j) as (stored tile, transpose flag)."""
    return ((A, i, j), N_) if trans == N_ else ((A, j, i), trans)


def _prec_of(M):
    return M.prec


# ----------------------------------------------------------------------------- TRSM
def trsm_program(ctx, side, uplo, trans, diag, alpha, A, B, prog=None, name="trsm"):
    prog = prog or TileProgram(ctx, name)
    prog.flops += flops(B.prec, "trsm", side == dplasmaLeft, B.m, B.n)
    if alpha != 1.0:
        s = prog.stage("scale")
        for (m, n) in _all_tiles(B):
            s.lascal((B, m, n), 0, alpha)
    if side == dplasmaLeft:
        lower_m = (uplo == dplasmaLower) == (trans == N_)
        order = list(range(B.mt)) if lower_m else list(range(B.mt - 1, -1, -1))
        for idx, k in enumerate(order):
            s1 = prog.stage(f"trsm_solve({k})")
            for n in range(B.nt):
                s1.trsm(side, uplo, trans, diag, 1.0, (A, k, k), (B, k, n))
            rest = order[idx + 1:]
            if rest:
                s2 = prog.stage(f"trsm_update({k})")
                for m in rest:
                    Mt, om = _op_tile(A, trans, m, k)
                    for n in range(B.nt):
                        s2.gemm((B, m, n), [(Mt, om, (B, k, n), N_)], alpha=-1.0, beta=1.0)
    else:
        upper_m = (uplo == dplasmaUpper) == (trans == N_)
        order = list(range(B.nt)) if upper_m else list(range(B.nt - 1, -1, -1))
        for idx, k in enumerate(order):
            s1 = prog.stage(f"trsm_solve({k})")
            for m in range(B.mt):
                s1.trsm(side, uplo, trans, diag, 1.0, (A, k, k), (B, m, k))
            rest = order[idx + 1:]
            if rest:
                s2 = prog.stage(f"trsm_update({k})")
                for n in rest:
                    Mt, om = _op_tile(A, trans, k, n)
                    for m in range(B.mt):
                        s2.gemm((B, m, n), [((B, m, k), N_, Mt, om)], alpha=-1.0, beta=1.0)
    return prog


def _all_tiles(M):
    return [(m, n) for n in range(M.nt) for m in range(M.mt)]


def trsm_New(ctx, side, uplo, trans, diag, alpha, A, B):
    return trsm_program(ctx, side, uplo, trans, diag, alpha, A, B).compile()


def trsm(ctx, side, uplo, trans, diag, alpha, A, B):
    return trsm_New(ctx, side, uplo, trans, diag, alpha, A, B).execute(ctx)


# ----------------------------------------------------------------------------- helpers: masked diagonal copies
def _tri_diag_copy(prog, A, uplo, diag, Tri, name="tri"):
    """Tri(k,k) := triangle(A(k,k)) (zeros elsewhere, unit diagonal if asked)."""
    s = prog.stage(name + "_zero")
    kt = min(A.mt, A.nt)
    for k in range(kt):
        s.laset((Tri, k, k), 0, 0.0, 0.0)
    s = prog.stage(name + "_copy")
    for k in range(kt):
        s.copy((A, k, k), (Tri, k, k), part=P_LOWER if uplo == dplasmaLower else P_UPPER)
    if diag == dplasmaUnit:
        s = prog.stage(name + "_unit")
        for k in range(kt):
            s.laset((Tri, k, k), P_DIAG, 0.0, 1.0)


def _sym_diag_copy(prog, A, uplo, Sym, trans_other, name="sym"):
    """Sym(k,k) := full symmetric (trans_other = T) / Hermitian (C) tile from A's uplo triangle."""
    kt = min(A.mt, A.nt)
    s = prog.stage(name + "_copy")
    for k in range(kt):
        s.copy((A, k, k), (Sym, k, k), part=P_LOWER if uplo == dplasmaLower else P_UPPER)
    s = prog.stage(name + "_mirror")
    for k in range(kt):
        s.copy((A, k, k), (Sym, k, k), part=P_SUPPER if uplo == dplasmaLower else P_SLOWER, trans=trans_other)
    if trans_other == C_ and A.dtype.is_complex:
        # Hermitian: the imaginary parts of the diagonal are taken as zero (BLAS zhemm / zherk semantics):
        # diag := (diag + conj(diag)) / 2
        s = prog.stage(name + "_realdiag")
        for k in range(kt):
            s.geadd((Sym, k, k), (Sym, k, k), 0.5, 0.5, part=P_DIAG, trans=C_)


# ----------------------------------------------------------------------------- TRMM
def trmm_New(ctx, side, uplo, trans, diag, alpha, A, B):
    """B := alpha op(A) B (left) or alpha B op(A) (right), A triangular."""
    prog = TileProgram(ctx, "trmm")
    prog.flops = flops(B.prec, "trmm", side == dplasmaLeft, B.m, B.n)
    Tri = A.like(name="Atri")
    W = B.like(name="W")
    _tri_diag_copy(prog, A, uplo, diag, Tri)
    s = prog.stage("trmm_products")
    lower_a = uplo == dplasmaLower
    for (m, n) in _all_tiles(B):
        terms = []
        if side == dplasmaLeft:
            # W(m,n) = sum_k op(A)(m,k) B(k,n); op(A) lower iff lower_a == (trans == N)
            lower_m = lower_a == (trans == N_)
            ks = range(0, m + 1) if lower_m else range(m, B.mt)
            for k in ks:
                if k == m:
                    terms.append(((Tri, m, m), trans, (B, k, n), N_))
                else:
                    Mt, om = _op_tile(A, trans, m, k)
                    terms.append((Mt, om, (B, k, n), N_))
        else:
            # W(m,n) = sum_k B(m,k) op(A)(k,n)
            upper_m = (not lower_a) == (trans == N_)
            ks = range(0, n + 1) if upper_m else range(n, B.nt)
            for k in ks:
                if k == n:
                    terms.append(((B, m, k), N_, (Tri, n, n), trans))
                else:
                    Mt, om = _op_tile(A, trans, k, n)
                    terms.append(((B, m, k), N_, Mt, om))
        s.gemm((W, m, n), terms, alpha=alpha, beta=0.0)
    s = prog.stage("trmm_copyback")
    for (m, n) in _all_tiles(B):
        s.copy((W, m, n), (B, m, n))
    tp = prog.compile()
    tp._keep = (Tri, W)
    return tp


def trmm(ctx, side, uplo, trans, diag, alpha, A, B):
    return trmm_New(ctx, side, uplo, trans, diag, alpha, A, B).execute(ctx)


# ----------------------------------------------------------------------------- SYMM / HEMM
def _symm_New(ctx, side, uplo, alpha, A, B, beta, C, herm):
    prog = TileProgram(ctx, "hemm" if herm else "symm")
    prog.flops = flops(C.prec, "hemm" if herm else "symm", side == dplasmaLeft, C.m, C.n)
    Sym = A.like(name="Asym")
    other = C_ if herm else T_
    _sym_diag_copy(prog, A, uplo, Sym, other)
    lower = uplo == dplasmaLower

    def afull(i, j):
        if i == j:
            return (Sym, i, i), N_
        if (i > j) == lower:
            return (A, i, j), N_
        return (A, j, i), other
    s = prog.stage("symm")
    for (m, n) in _all_tiles(C):
        terms = []
        if side == dplasmaLeft:
            for k in range(A.mt):
                t, o = afull(m, k)
                terms.append((t, o, (B, k, n), N_))
        else:
            for k in range(A.nt):
                t, o = afull(k, n)
                terms.append(((B, m, k), N_, t, o))
        s.gemm((C, m, n), terms, alpha=alpha, beta=beta)
    tp = prog.compile()
    tp._keep = (Sym,)
    return tp


def symm_New(ctx, side, uplo, alpha, A, B, beta, C):
    return _symm_New(ctx, side, uplo, alpha, A, B, beta, C, herm=False)


def hemm_New(ctx, side, uplo, alpha, A, B, beta, C):
    return _symm_New(ctx, side, uplo, alpha, A, B, beta, C, herm=True)


def symm(ctx, side, uplo, alpha, A, B, beta, C):
    return symm_New(ctx, side, uplo, alpha, A, B, beta, C).execute(ctx)


def hemm(ctx, side, uplo, alpha, A, B, beta, C):
    return hemm_New(ctx, side, uplo, alpha, A, B, beta, C).execute(ctx)


# ----------------------------------------------------------------------------- SYRK / HERK / SYR2K / HER2K
def _tri_tiles(C, uplo):
    return [(m, n) for (m, n) in _all_tiles(C) if (m >= n if uplo == dplasmaLower else m <= n)]


def _rank_k_New(ctx, uplo, trans, alpha, A, B, beta, C, herm, two):
    name = ("her2k" if herm else "syr2k") if two else ("herk" if herm else "syrk")
    prog = TileProgram(ctx, name)
    kdim = A.n if trans == N_ else A.m
    prog.flops = flops(C.prec, name, kdim, C.n)
    tr = C_ if herm else T_
    mask = MASK_LOWER if uplo == dplasmaLower else MASK_UPPER
    kt = A.nt if trans == N_ else A.mt

    def terms_for(X, Y, m, n):
        out = []
        for k in range(kt):
            if trans == N_:
                out.append(((X, m, k), N_, (Y, n, k), tr))
            else:
                out.append(((X, k, m), tr, (Y, k, n), N_))
        return out
    s = prog.stage(name)
    for (m, n) in _tri_tiles(C, uplo):
        s.gemm((C, m, n), terms_for(A, B if two else A, m, n), alpha=alpha, beta=beta,
               mask=mask if m == n else 0)
    if two:
        a2 = alpha.conjugate() if (herm and isinstance(alpha, complex)) else alpha
        s = prog.stage(name + "_2")
        for (m, n) in _tri_tiles(C, uplo):
            s.gemm((C, m, n), terms_for(B, A, m, n), alpha=a2, beta=1.0, mask=mask if m == n else 0)
    return prog.compile()


def syrk_New(ctx, uplo, trans, alpha, A, beta, C):
    return _rank_k_New(ctx, uplo, trans, alpha, A, None, beta, C, herm=False, two=False)


def herk_New(ctx, uplo, trans, alpha, A, beta, C):
    return _rank_k_New(ctx, uplo, trans, alpha, A, None, beta, C, herm=True, two=False)


def syr2k_New(ctx, uplo, trans, alpha, A, B, beta, C):
    return _rank_k_New(ctx, uplo, trans, alpha, A, B, beta, C, herm=False, two=True)


def her2k_New(ctx, uplo, trans, alpha, A, B, beta, C):
    return _rank_k_New(ctx, uplo, trans, alpha, A, B, beta, C, herm=True, two=True)


def syrk(ctx, uplo, trans, alpha, A, beta, C):
    return syrk_New(ctx, uplo, trans, alpha, A, beta, C).execute(ctx)


def herk(ctx, uplo, trans, alpha, A, beta, C):
    return herk_New(ctx, uplo, trans, alpha, A, beta, C).execute(ctx)


def syr2k(ctx, uplo, trans, alpha, A, B, beta, C):
    return syr2k_New(ctx, uplo, trans, alpha, A, B, beta, C).execute(ctx)


def her2k(ctx, uplo, trans, alpha, A, B, beta, C):
    return her2k_New(ctx, uplo, trans, alpha, A, B, beta, C).execute(ctx)


# ----------------------------------------------------------------------------- GER
def gerc_New(ctx, alpha, X, Y, A):
    """A := alpha x y^H + A (dplasma_zgerc_New, src/zger.jdf): X is M x 1, Y is N x 1 -- a K = 1 GEMM."""
    from .gemm import gemm_New
    return gemm_New(ctx, dplasmaNoTrans, dplasmaConjTrans if A.dtype.is_complex else dplasmaTrans, alpha, X, Y, 1.0,
                    A, name="ger")


def geru_New(ctx, alpha, X, Y, A):
    """A := alpha x y^T + A (dplasma_zgeru_New)."""
    from .gemm import gemm_New
    return gemm_New(ctx, dplasmaNoTrans, dplasmaTrans, alpha, X, Y, 1.0, A, name="ger")


def gerc(ctx, alpha, X, Y, A):
    gerc_New(ctx, alpha, X, Y, A).execute(ctx)
    return 0


def geru(ctx, alpha, X, Y, A):
    geru_New(ctx, alpha, X, Y, A).execute(ctx)
    return 0
