"""Stacked-domain Householder QR: the MI355X engine of geqrf / geqrf_param on 1 x Q grids.

Reference: ``src/zgeqrf.jdf`` (flat TS tree: zgeqrt(k) :98, zunmqr(k,n) :198, ztsqrt(k,m) :314,
ztsmqr(k,m,n) :443), ``src/zgeqrf_param.jdf`` (trees: TS domains + TT kills), ``src/zunmqr_*.jdf``,
``src/zungqr*.jdf``.

Why a different kernel decomposition than the tile DAG of models/qr.py: a TS chain (GEQRT on
the head, then TSQRT of every row of the domain, one after the other) is a sequence of
single-workgroup, column-at-a-time kernels -- latency bound on a 256-CU part (measured: 2.6 ms
per 256-column TSQRT launch, 54-60 % of a 16k factorisation, profiles/README.md).  Here a TS
domain is factored as ONE stacked tall panel by a persistent kernel that spreads the rows over
every CU (ops.qr_panel -> csrc/kernels/qr_panel.hip), and its trailing update is three batched
MFMA GEMM launches of the whole remaining matrix:

    W = V^T C   (split over the domain rows, partials summed)     W' = T^T W     C -= V W'

Storage format (what unmqr / ungqr / geqrs / gels of this package consume; real precisions):
  * every TS domain D = [h, m1, m2, ...] of panel k (the head and the rows it TS-kills, in kill
    order) -- for the flat tree the whole panel -- holds the Householder QR of the stacked rows
    [A(h,k); A(m1,k); ...]: R in the upper triangle of A(h,k), V below the diagonal of A(h,k)
    and in the full tiles A(m_i,k) (LAPACK dgeqrf layout for the domain); TS(h,k) holds the
    IB x IB diagonal blocks of the domain's compact-WY T (LAPACK dgeqrt's T layout);
  * every TT kill (p, m) of the tree is the Householder QR of the stacked R factors [R_p; R_m]:
    R into A(p,k)'s upper triangle, V2 (upper triangular) into A(m,k)'s upper triangle, T blocks
    in TT(m,k) -- the same places the reference's TTQRT uses;
  * per panel, all domains come first, then the TT kills in plan order.
The full T of a reflector set is rebuilt from V and its diagonal blocks when Q is applied.

1 x Q grids (single-domain plans): the owner of panel column k factors it and broadcasts V and T
along the process row (RCCL); every rank applies them to its own columns.  For Q-side applications
from the right the partial W = C V is all-reduced along the row.

Lookahead (single-domain trees, e.g. the flat tree or HQR with one domain per process row):
the panel stream factors panel k+1 right after applying Q_k^T to column k+1, while the update
stream applies Q_k^T to columns k+2.. (the reference's priority-driven lookahead, done with
two HIP streams of different priority).
"""
from __future__ import annotations

import contextlib
import os

import numpy as np
import torch

from ..constants import dplasmaConjTrans, dplasmaLeft, dplasmaNoTrans, dplasmaTrans
from ..ops import tile_ops as ops
from ..ops.batch import GemmBatch, TileBatch, unpredicated
from ..parallel import comm
from ..runtime.taskpool import Taskpool
from ..utils.flops import flops
from . import qrtree

# T_ is the adjoint: V^H / T^H for complex (the GEMM engine treats ConjTrans as Trans for real types)
N_, T_ = dplasmaNoTrans, dplasmaConjTrans
PART_FULL, PART_UPPER, PART_SLOWER, PART_DIAG = 0, 2, 3, 5

_ENGINE = [os.environ.get("DPLASMA_QR_ENGINE", "panel")]


@contextlib.contextmanager
def engine(name: str):
    """Temporarily select the QR engine ("panel" or "tile") -- tests use it to run the tile
    algorithm on one process as the reference of a distributed run."""
    old = _ENGINE[0]
    _ENGINE[0] = name
    try:
        yield
    finally:
        _ENGINE[0] = old


def _rup(x, m):
    return (x + m - 1) // m * m


# ----------------------------------------------------------------------------- plans
def step_plan(tree, k, merge=False, prow=None):
    """(domains, tt_stacks) of panel k: domains = [[head, ts victims...], ...], tt_stacks =
    [(p, [m, ...]), ...]; None when a TS kill's pivot is not a head (not expressible as stacked
    domains).

    merge=False: one stack per TT kill (p, [m]) in the tree's kill order.  merge=True (one process
    row): the step's TT kills reduce every domain head to one survivor, so the whole TT subtree is
    factored as ONE stacked panel of triangles [R_root; R_m1; R_m2; ...] (victims in kill order),
    the way a TS domain is one stacked panel: V stays upper triangular in each victim's tile, R
    lands in the survivor's, one T for the stack.  Mathematically the same reduction (an
    orthogonal Q, the same R up to row signs); what changes is the launch count -- the trees are
    shaped for a tile DAG that pipelines kills across panels, and executed round by round their
    depth is paid in launches (the greedy tree at 32k, a = 4: up to 15 dependent rounds per step,
    1864 panel launches in all; merged: 2 per step).  A kill set without a unique survivor falls
    back to one stack per pivot at level 1 + its deepest victim's level.  Stacks come in level order."""
    heads = list(tree.heads(k))
    doms = {h: [h] for h in heads}
    kills = []
    for (p, m, t) in tree.kills(k):
        if t == qrtree.KILLED_BY_TS:
            if p not in doms:
                return None
            doms[p].append(m)
        else:
            kills.append((p, m))
    if not merge:
        return [doms[h] for h in heads], [(p, [m]) for (p, m) in kills]
    if merge == "row":
        return [doms[h] for h in heads], _row_stacks(kills, prow)
    victims = [m for (_, m) in kills]
    roots = {p for (p, _) in kills} - set(victims)
    if len(roots) == 1:
        return [doms[h] for h in heads], [(roots.pop(), victims)]
    stacks, order = {}, []
    for (p, m) in kills:
        if p not in stacks:
            stacks[p] = []
            order.append(p)
        stacks[p].append(m)
    lev = {}

    def level(x):
        if x not in stacks:
            return 0
        if x not in lev:
            lev[x] = 1 + max(level(m) for m in stacks[x])
        return lev[x]
    rank = {p: i for i, p in enumerate(order)}
    tts = sorted(((p, stacks[p]) for p in order), key=lambda e: (level(e[0]), rank[e[0]]))
    return [doms[h] for h in heads], tts


def _row_stacks(kills, prow):
    """merge="row" (trees over several process rows): the kills inside one process row become stacked panels
    -- every local subtree of a step is ONE stack [R_root; R_v1; R_v2; ...] factored by the row's owner of the
    panel column, the one-process-row trick applied per row -- while the kills that cross process rows stay
    pairwise (R / V2 / T and the partial W exchanged between the two rows).  Kills are taken in tree order; a
    local kill whose victim leads an open stack absorbs that stack (its triangles join the killer's stack
    unreduced: the same QR of the union), and a cross-row kill first closes (emits) the open stacks of both
    its tiles, so every entry sees its tiles' R as the tree order has them.  The trees' low-level rounds
    inside a row (greedy at 2 x 4: up to ~6 per step) collapse to one launch; src/dplasma_hqr.c:1670-1948
    lays out the same two-level reduction (local trees, then the distributed high-level tree)."""
    open_, order, out = {}, [], []

    def close(x):
        if x in open_:
            out.append((x, open_.pop(x)))
            order.remove(x)
    for (p, m) in kills:
        if prow(p) == prow(m):
            vict = [m] + (open_.pop(m) if m in open_ else [])
            if m in order:
                order.remove(m)
            if p in open_:
                open_[p] += vict
            else:
                open_[p] = vict
                order.append(p)
        else:
            close(p)
            close(m)
            out.append((p, [m]))
    for x in list(order):
        close(x)
    return out


def _merge_tt(A, tree):
    """How a step's TT kills are grouped: one process row and a one-row tree -> every pivot's kills one
    stack (True); several process rows (a P x Q grid, or one process running a tree built for p rows, which
    must lay its factors out as the grid run does) -> stacks per process row, cross-row kills pairwise
    ("row"); DPLASMA_QR_MERGE_TT=0 keeps every kill pairwise, =1 limits merging to one-row trees."""
    env = os.environ.get("DPLASMA_QR_MERGE_TT", "row")
    if env == "0":
        return False
    if A.grid.P == 1 and int(getattr(tree, "p", 1) or 1) == 1:
        return True
    return "row" if env == "row" else False


def _tree_prow(A, tree):
    """Process row of tile row m as the step plans see it: the grid's (P > 1), else the tree's p rows."""
    if A.grid.P > 1:
        return lambda m: _prow(A, m)
    p = max(1, int(getattr(tree, "p", 1) or 1))
    return lambda m: m % p


def _plan(A, tree, k):
    return step_plan(tree, k, _merge_tt(A, tree), _tree_prow(A, tree))


def _prow(A, m):
    return A.grid.prow(m + A.it0)


def usable(A, tree=None) -> bool:
    """The stacked-domain engine handles this factorisation (and therefore owns its format)."""
    if _ENGINE[0] != "panel":
        return False
    if A.dtype not in (torch.float32, torch.float64, torch.complex64, torch.complex128):
        return False
    if A.grid.kq != 1 or A.mb != A.nb or A.nb > ops.QR_PANEL_MAXW:
        return False
    if A.device.type == "cuda" and A.m > ops.qr_panel_max_rows(A.device):
        return False
    if tree is not None:
        plans = [step_plan(tree, k) for k in range(min(A.mt, A.nt))]
        if any(p is None for p in plans):
            return False
        # distributed grids: every TS domain lives on one process row (its owner factors it with no
        # communication); TT kills may cross process rows (exchange of R / V2 / partial W)
        if A.grid.P > 1 and any(len({_prow(A, r) for r in d}) != 1 for dd, _ in plans for d in dd):
            return False
    return True


def _sequence(A, tree):
    """Factorisation order: [("dom", k, rows) | ("tt", k, p, [m, ...])] over all panels."""
    seq = []
    for k in range(min(A.mt, A.nt)):
        doms, tts = _plan(A, tree, k)
        seq += [("dom", k, d) for d in doms]
        seq += [("tt", k, p, ms) for (p, ms) in tts]
    return seq


# ----------------------------------------------------------------------------- batched updates
def _offsets(C, rows, cols):
    """off[i, j] = C.offset(rows[i], cols[j]) (tile offsets are additive in row and column)."""
    rows, cols = list(rows), list(cols)
    R = np.array([C.offset(r, cols[0]) for r in rows], dtype=np.int64)
    Cc = np.array([C.offset(rows[0], n) for n in cols], dtype=np.int64) - R[0]
    return R[:, None] + Cc[None, :]


# W = V^T C is split over S row groups (partials summed) until a launch has about this many
# 128 x 128 output workgroups (DPLASMA_QR_SPLIT_WG)
QR_SPLIT_TARGET_WG = int(os.environ.get("DPLASMA_QR_SPLIT_WG", 512))


class _Left:
    """C(rows, cols) := op(Q)^T-style block reflector application from the left:
    W = V^T C (split over S row groups, partials summed), W' = op(T) W, C -= V W'.
    Batches are built with whole-array numpy operations (millions of tiles at 64k)."""

    def __init__(self, C, rows, voff, kf, cols, target_wg=None):
        self.kf = kf
        if target_wg is None:
            target_wg = QR_SPLIT_TARGET_WG
        self.empty = not cols or not rows
        self.S, self.wlen = 1, 0
        if self.empty:
            return
        rows, cols = list(rows), list(cols)
        voff = np.asarray(voff, dtype=np.int64)
        hr = np.array([C.tile_rows(r) for r in rows], dtype=np.int64)
        wn = np.array([C.tile_cols(n) for n in cols], dtype=np.int64)
        woff = kf * np.concatenate([[0], np.cumsum(wn)[:-1]])
        self.wlen = int(wn.sum()) * kf
        nrow, ncol = len(rows), len(cols)
        off = _offsets(C, rows, cols)
        wg = max(1, ncol * max(1, kf // 128) * max(1, C.nb // 128))
        self.S = S = max(1, min(nrow, -(-target_wg // wg)))
        g1, g2, g3 = GemmBatch(), GemmBatch(), GemmBatch()
        grps = np.array_split(np.arange(nrow), S)
        g1.add_arrays((np.arange(S, dtype=np.int64)[:, None] * self.wlen + woff[None, :]).ravel(), kf, np.tile(wn, S),
                      np.repeat([len(g) for g in grps], ncol),
                      np.concatenate([np.tile(voff[g], ncol) for g in grps]),
                      np.concatenate([off[g, :].T.ravel() for g in grps]),
                      np.concatenate([np.tile(hr[g], ncol) for g in grps]))
        g2.add_arrays(woff, kf, wn, 1, 0, woff, kf)
        g3.add_arrays(off.T.ravel(), np.tile(hr, ncol), np.repeat(wn, nrow), 1, np.tile(voff, ncol),
                      np.repeat(woff, nrow), kf)
        self.g1, self.g2, self.g3 = g1.finalize(), g2.finalize(), g3.finalize()

    def run(self, C, V, ldv, Tm, ldt, Wp, W, W2, qt: bool, group=None, reduce=None):
        if self.empty:
            return
        kf, L = self.kf, self.wlen
        ops.gemm(T_, N_, 1.0, V, ldv, C.data, C.ld, 0.0, Wp, kf, self.g1)
        if self.S > 1:
            ops.sum_partials(Wp, L, self.S, L, W)
            src = W
        else:
            src = Wp
        if reduce is not None:   # reflector rows split over two process rows: add the partner's part
            reduce(src[:L])
        ops.gemm(T_ if qt else N_, N_, 1.0, Tm, ldt, src, kf, 0.0, W2, kf, self.g2)
        ops.gemm(N_, N_, -1.0, V, ldv, W2, kf, 1.0, C.data, C.ld, self.g3)


class _LeftMulti:
    """The _Left application of several reflector sets on disjoint row sets at once (the TS domains of
    one panel step, or the TT stacks of one tree round): three GEMM launches for the whole group.
    parts: (rows, voff (element offsets of each row tile in the V buffer), wbase (offset of the part's
    W block), tbase (offset of its T in the T buffer)); every part has kf reflectors."""

    def __init__(self, C, parts, kf, cols):
        self.kf = kf
        cols = list(cols)
        self.empty = not cols or not parts
        self.wlen = 0
        if self.empty:
            return
        wn = np.array([C.tile_cols(n) for n in cols], dtype=np.int64)
        wloc = kf * np.concatenate([[0], np.cumsum(wn)[:-1]])
        ncol = len(cols)
        g1, g2, g3 = GemmBatch(), GemmBatch(), GemmBatch()
        for rows, voff, wbase, tbase in parts:
            rows = list(rows)
            voff = np.asarray(voff, dtype=np.int64)
            hr = np.array([C.tile_rows(r) for r in rows], dtype=np.int64)
            nrow = len(rows)
            off = _offsets(C, rows, cols)
            woff = wbase + wloc
            g1.add_arrays(woff, kf, wn, nrow, np.tile(voff, ncol), off.T.ravel(), np.tile(hr, ncol))
            g2.add_arrays(woff, kf, wn, 1, tbase, woff, kf)
            g3.add_arrays(off.T.ravel(), np.tile(hr, ncol), np.repeat(wn, nrow), 1, np.tile(voff, ncol),
                          np.repeat(woff, nrow), kf)
            self.wlen = max(self.wlen, int(wbase + kf * wn.sum()))
        self.g1, self.g2, self.g3 = g1.finalize(), g2.finalize(), g3.finalize()

    def run(self, C, V, ldv, Tm, ldt, W, W2, qt: bool, Yv=None):
        """Yv (optional) = V op(T), formed once per reflector set: C -= Yv (V^T C) -- two GEMM launches,
        and no T^T W product whose cost grows with the trailing width (9 % of an a = 4 HQR step's flops)."""
        if self.empty:
            return
        kf = self.kf
        ops.gemm(T_, N_, 1.0, V, ldv, C.data, C.ld, 0.0, W, kf, self.g1)
        if Yv is not None:
            ops.gemm(N_, N_, -1.0, Yv, ldv, W, kf, 1.0, C.data, C.ld, self.g3)
            return
        ops.gemm(T_ if qt else N_, N_, 1.0, Tm, ldt, W, kf, 0.0, W2, kf, self.g2)
        ops.gemm(N_, N_, -1.0, V, ldv, W2, kf, 1.0, C.data, C.ld, self.g3)


class _Right:
    """C(rows, cols) := C op(Q) (cols = the reflector rows): W = C V, W' = W op(T), C -= W' V^T."""

    def __init__(self, C, crows, vcols, voff, kf, target_wg=None, split=True):
        self.kf = kf
        if target_wg is None:
            target_wg = QR_SPLIT_TARGET_WG
        crows, vcols = list(crows), list(vcols)
        hc = np.array([C.tile_rows(i) for i in crows], dtype=np.int64)
        roff = np.concatenate([[0], np.cumsum(hc)[:-1]]).astype(np.int64)
        self.ldw = max(1, _rup(int(hc.sum()), 16))
        self.wlen = self.ldw * kf
        self.empty = not crows or not vcols
        self.nocols = not vcols
        self.S = 1
        if self.empty:
            return
        voff = np.asarray(voff, dtype=np.int64)
        wc = np.array([C.tile_cols(n) for n in vcols], dtype=np.int64)
        ncol, nrow = len(vcols), len(crows)
        off = _offsets(C, crows, vcols)
        wg = max(1, nrow * max(1, kf // 128) * max(1, C.mb // 128))
        self.S = S = max(1, min(ncol, -(-target_wg // wg))) if split else 1
        g1, g2, g3 = GemmBatch(), GemmBatch(), GemmBatch()
        grps = np.array_split(np.arange(ncol), S)
        g1.add_arrays((np.arange(S, dtype=np.int64)[:, None] * self.wlen + roff[None, :]).ravel(), np.tile(hc, S), kf,
                      np.repeat([len(g) for g in grps], nrow),
                      np.concatenate([off[:, g].ravel() for g in grps]),
                      np.concatenate([np.tile(voff[g], nrow) for g in grps]),
                      np.concatenate([np.tile(wc[g], nrow) for g in grps]))
        g2.add_arrays(roff, hc, kf, 1, roff, 0, kf)
        g3.add_arrays(off.ravel(), np.repeat(hc, ncol), np.tile(wc, nrow), 1, np.repeat(roff, ncol),
                      np.tile(voff, nrow), kf)
        self.g1, self.g2, self.g3 = g1.finalize(), g2.finalize(), g3.finalize()

    def run(self, C, V, ldv, Tm, ldt, Wp, W, W2, qt: bool, group=None):
        kf, L, ldw = self.kf, self.wlen, self.ldw
        if group is not None:
            # 1 x Q grid: the reflector rows are C's columns, spread over the process row
            if self.nocols:
                Wp[:L].zero_()
            else:
                ops.gemm(N_, N_, 1.0, C.data, C.ld, V, ldv, 0.0, Wp, ldw, self.g1)
            comm.allreduce(Wp[:L], group=group)
            if self.empty:
                return
            ops.gemm(N_, T_ if qt else N_, 1.0, Wp, ldw, Tm, ldt, 0.0, W2, ldw, self.g2)
            ops.gemm(N_, T_, -1.0, W2, ldw, V, ldv, 1.0, C.data, C.ld, self.g3)
            return
        if self.empty:
            return
        ops.gemm(N_, N_, 1.0, C.data, C.ld, V, ldv, 0.0, Wp, ldw, self.g1)
        if self.S > 1:
            ops.sum_partials(Wp, L, self.S, L, W)
            src = W
        else:
            src = Wp
        ops.gemm(N_, T_ if qt else N_, 1.0, src, ldw, Tm, ldt, 0.0, W2, ldw, self.g2)
        ops.gemm(N_, T_, -1.0, W2, ldw, V, ldv, 1.0, C.data, C.ld, self.g3)


def _work_buffers(updates, dtype, device):
    """Wp (split partials), W (their sum), W2 sized for a list of _Left/_Right plans."""
    n1 = max([u.S * u.wlen for u in updates] + [1])
    n2 = max([u.wlen for u in updates] + [1])
    z = lambda n: torch.zeros(n, dtype=dtype, device=device)  # noqa: E731
    return z(n1), z(n2), z(n2)


# ----------------------------------------------------------------------------- T storage
def _store_T(Tm, ldt, kf, Td, row, k):
    """Diagonal IB x IB blocks of the kf x kf T into tile Td(row, k) (dgeqrt layout)."""
    ib = Td.mb
    base, ld = Td.offset(row, k), Td.ld
    nfull = kf // ib
    if nfull:
        src = torch.as_strided(Tm, (nfull, ib, ib), (ib * ldt + ib, 1, ldt), 0)
        dst = torch.as_strided(Td.data, (nfull, ib, ib), (ib * ld, 1, ld), base)
        dst.copy_(src)
    r = kf - nfull * ib
    if r:
        c0 = nfull * ib
        src = torch.as_strided(Tm, (r, r), (1, ldt), c0 * ldt + c0)
        torch.as_strided(Td.data, (r, r), (1, ld), base + c0 * ld).copy_(src)


def _keep_full_T(Tm, ldt, kf, Td, row, k):
    """Keep the whole compact-WY T of a factored domain / TT stack next to its reference-layout
    diagonal blocks (Td.full_T[(row, k)], nb x nb per panel: 2 MiB at NB = 512), so the apply
    (unmqr / ungqr / geqrs / gels) reuses it instead of rebuilding the coupling blocks."""
    store = getattr(Td, "full_T", None)
    if store is None:
        store = Td.full_T = {}
    t = store.get((row, k))
    if t is None or t.numel() < kf * kf or t.device != Tm.device:
        t = store[(row, k)] = torch.empty(kf * kf, dtype=Tm.dtype, device=Tm.device)
    t[: kf * kf].view(kf, kf).t().copy_(torch.as_strided(Tm, (kf, kf), (1, ldt), 0))  # t may be a view


def _rebuild_T(V, ldv, M, kf, Td, row, k, out, ldt):
    """Full compact-WY T: the copy kept by the factorisation when there is one, else rebuilt from
    the stored diagonal IB blocks and V (coupling T12 = -T11 (V1^H V2) T22, block column by block
    column) with the batched MFMA GEMM engine -- no vendor BLAS on the device path."""
    kept = getattr(Td, "full_T", {}).get((row, k))
    dst = torch.as_strided(out, (kf, kf), (1, ldt), 0)
    if kept is not None and kept.device == out.device and kept.numel() >= kf * kf:
        dst.copy_(kept[: kf * kf].view(kf, kf).t())  # kept may be a view (batched factorisation)
        return
    ib = Td.mb
    dst.zero_()
    for b0 in range(0, kf, ib):
        bs = min(ib, kf - b0)
        dst[b0:b0 + bs, b0:b0 + bs] = torch.triu(Td.tile(row, k)[:bs, b0:b0 + bs])
    if kf <= ib:
        return
    ct = dplasmaConjTrans if V.dtype.is_complex else dplasmaTrans
    G = torch.empty(kf * kf, dtype=V.dtype, device=V.device)   # G = V^H V  (kf x kf, ld kf)
    X = torch.empty(kf * ib, dtype=V.dtype, device=V.device)   # X = T(:b0, :b0) G(:b0, b0:b0+bs)
    gb = GemmBatch()
    gb.add(0, kf, kf, [(0, 0, M)])
    ops.gemm(ct, N_, 1.0, V, ldv, V, ldv, 0.0, G, kf, gb)
    for b0 in range(ib, kf, ib):
        bs = min(ib, kf - b0)
        g1 = GemmBatch()
        g1.add(0, b0, bs, [(0, b0 * kf, b0)])                  # X = T11 G(:b0, b0:)
        ops.gemm(N_, N_, 1.0, out, ldt, G, kf, 0.0, X, b0, g1)
        g2 = GemmBatch()
        g2.add(b0 * ldt, b0, bs, [(0, b0 + b0 * ldt, bs)])     # T(:b0, b0:) = -X T22
        ops.gemm(N_, N_, -1.0, X, b0, out, ldt, 0.0, out, ldt, g2)


# ----------------------------------------------------------------------------- factorisation
class _Factor:
    def __init__(self, ctx, A, TS, TT, tree, inplace=True):
        self.ctx, self.A, self.TS, self.TT = ctx, A, TS, TT
        # inplace=False: every domain is gathered into the panel buffer, none factored in place in A (a caller
        # that issues the panel kernels beside a predicate they ignore -- models/lu_qr.py -- needs A untouched)
        self.inplace = inplace
        dev, dt = A.device, A.dtype
        nb = A.nb
        self.kt = min(A.mt, A.nt)
        # distributed: V and T travel along the process row(s) of the reflector rows (RCCL);
        # TT kills across process rows exchange R / V2 / T and the partial W between the two rows
        self.dist = ctx.world > 1
        self.plans = [_plan(A, tree, k) for k in range(self.kt)]
        for k, (doms, tts) in enumerate(self.plans):
            for d in doms:
                if TS.rank_of(d[0], k) != A.rank_of(d[0], k):
                    raise ValueError("geqrf: TS must be distributed like A (tile rows and columns)")
            for (pp, ms) in tts:
                if TT.rank_of(ms[0], k) != A.rank_of(ms[0], k):
                    raise ValueError("geqrf: TT must be distributed like A (tile rows and columns)")
        self.simple = all(len(d) == 1 and not t for d, t in self.plans) and A.grid.P == 1
        # one process, a tree with several domains / TT rounds per panel: every domain of a panel step in
        # ONE multi-panel launch and one batched update, then each TT round likewise (DPLASMA_QR_BATCHED=0:
        # entry by entry)
        self.batched = (not self.simple and not self.dist and A.grid.P == 1 and A.grid.Q == 1
                        and os.environ.get("DPLASMA_QR_BATCHED", "1") != "0")
        if self.batched:
            self._init_batched()
            return
        self.ldp = max(16, _rup(A.m, 16))
        # general trees (several domains / TT kills per panel step, or P x Q grids): look-ahead like the
        # simple path -- every entry's update split into column k+1 (panel stream) and the rest (update
        # stream), so panel step k+1 overlaps the bulk update of step k; V / T per (step parity, entry)
        self.la = not self.simple and os.environ.get("DPLASMA_QR_LOOKAHEAD", "1") != "0"
        nent = max([len(d) + len(t) for d, t in self.plans] + [1])
        nbuf = 2 if self.simple else (2 * nent if self.la else 1)
        self.nent = nent
        self.P = [torch.zeros(self.ldp * nb, dtype=dt, device=dev) for _ in range(1 if self.la else nbuf)]
        self.V = [torch.zeros(self.ldp * nb, dtype=dt, device=dev) for _ in range(nbuf)]
        self.Tm = [torch.zeros(nb * nb, dtype=dt, device=dev) for _ in range(nbuf)]
        self.R = torch.zeros(nb * nb, dtype=dt, device=dev)     # cross-row TT: the partner's tile
        self.ws = ops.qr_panel_workspace(nb, nb, dt, dev)
        self.info = torch.zeros(1, dtype=torch.int32, device=dev)
        self.steps = [self._build(k) for k in range(self.kt)]
        # VSEND (look-ahead on P x Q, DPLASMA_QR_VSEND=1): the broadcasts whose root is this rank run as a task of
        # their own after the step's panels (own stream) -- the root's next-column update does not wait for its V / T
        # to reach the row (every root of a step on one row communicator is that row's rank of the panel column, so
        # deferring all of them keeps each communicator's order).  Off by default: 2 x 4 64k rank replay 41.1 % with,
        # 43.6 % without (profiles/r6_hqr_config4.txt)
        self.vsend_task = (self.la and self.dist and A.grid.Q > 1 and os.environ.get("DPLASMA_QR_VSEND", "0") == "1")
        self._vq, self._cur_k = {}, None
        if self.vsend_task and dev.type == "cuda" and "vsend" not in ctx.streams:
            ctx.streams["vsend"] = torch.cuda.Stream(device=dev, priority=torch.cuda.Stream.priority_range()[1])
        ups = [u for st in self.steps for e in st for u in (e.get("next"), e.get("rest"), e.get("upd")) if u]
        if self.simple or self.la:
            nx = [e["next"] for st in self.steps for e in st if e.get("next")]
            rs = [e["rest"] for st in self.steps for e in st if e.get("rest")]
            self.wn = _work_buffers(nx, dt, dev)
            self.wr = _work_buffers(rs, dt, dev)
            self.xtmp_n = torch.zeros(max([u.wlen for u in nx] + [1]), dtype=dt, device=dev)
            self.xtmp = torch.zeros(max([u.wlen for u in rs] + [1]), dtype=dt, device=dev)
        else:
            self.wr = _work_buffers(ups, dt, dev)
            self.xtmp = torch.zeros(max([u.wlen for u in ups] + [1]), dtype=dt, device=dev)

    # ------------------------------------------------------------------ batched general trees (P == 1)
    def _init_batched(self):
        A, TS, TT = self.A, self.TS, self.TT
        dev, dt = A.device, A.dtype
        nb = A.nb
        ncu = torch.cuda.get_device_properties(dev).multi_processor_count if dev.type == "cuda" else 256
        specs = []
        for k in range(self.kt):
            doms, tts = self.plans[k]
            lev, rounds = {}, {}
            for (p_, ms) in tts:
                L = max([lev.get(p_, 0)] + [lev.get(m_, 0) for m_ in ms]) + 1
                lev[p_] = L
                rounds.setdefault(L, []).append([p_] + list(ms))
            cols = list(range(k + 1, A.nt))
            kgroups = []
            for kind, members in [("dom", doms)] + [("tt", rounds[L]) for L in sorted(rounds)]:
                ents = [self._entry(k, list(r), kind == "tt") for r in members]
                # launches that fit the CUs (every panel's workgroups co-resident), one kf per launch
                cur, g = [], 0
                for e in ents:
                    ge = -(-e["M"] // 256)
                    if cur and (g + ge > ncu or e["kf"] != cur[0]["kf"]):
                        kgroups.append((k, kind, cur, cols))
                        cur, g = [], 0
                    cur.append(e)
                    g += ge
                if cur:
                    kgroups.append((k, kind, cur, cols))
            specs.append(kgroups)
        # buffer sizes over every group
        need_p = need_v = need_w = need_t = 1
        ncol_el = lambda cols: sum(A.tile_cols(n) for n in cols)  # noqa: E731
        # V / T of every group of a step at their own offsets (look-ahead applies them after all the
        # step's panels); the gather buffer is reused group after group
        self._vt_base = []
        for kgroups in specs:
            vbase = tbase = 0
            bases = []
            for (k, kind, ents, cols) in kgroups:
                ld = max(e["ld"] for e in ents)
                bases.append((vbase, tbase))
                vbase += len(ents) * ld * nb
                tbase += len(ents) * nb * nb
                need_p = max(need_p, len(ents) * ld * nb)
                need_w = max(need_w, len(ents) * ents[0]["kf"] * max(1, ncol_el(cols)))
            self._vt_base.append(bases)
            need_v, need_t = max(need_v, vbase), max(need_t, tbase)
        # look-ahead (DPLASMA_QR_LOOKAHEAD, default on): every group's update is split into column k+1
        # (panel stream, right after the panels) and the rest (update stream), so the panel chain of step
        # k+1 -- the TS launch and every TT round -- overlaps the bulk update of step k; V / T double-buffered
        self.bla = os.environ.get("DPLASMA_QR_LOOKAHEAD", "1") != "0"
        nbuf = 2 if self.bla else 1
        self.Pb = torch.zeros(need_p, dtype=dt, device=dev)
        self.Vbs = [torch.zeros(need_v, dtype=dt, device=dev) for _ in range(nbuf)]
        # Y = V op(T) of every group (DPLASMA_QR_VT=0: apply T to W instead)
        self.use_vt = os.environ.get("DPLASMA_QR_VT", "1") != "0"
        self.Ybs = [torch.zeros(need_v, dtype=dt, device=dev) for _ in range(nbuf)] if self.use_vt else None
        self.Tbs = [torch.zeros(need_t, dtype=dt, device=dev) for _ in range(nbuf)]
        self.Wb = torch.zeros(need_w, dtype=dt, device=dev)
        self.W2b = torch.zeros(need_w, dtype=dt, device=dev)
        if self.bla:
            need_n = max([len(ents) * ents[0]["kf"] * nb for kg in specs for (_, _, ents, _) in kg] + [1])
            self.Wn = torch.zeros(need_n, dtype=dt, device=dev)
            self.W2n = torch.zeros(need_n, dtype=dt, device=dev)
        self.info = torch.zeros(1, dtype=torch.int32, device=dev)
        self.bsteps = [[self._group(*gspec, *self._vt_base[i][gi]) for gi, gspec in enumerate(kgroups)]
                       for i, kgroups in enumerate(specs)]

    def _group(self, k, kind, ents, cols, vbase=0, tbase=0):
        A = self.A
        nb, kb = A.nb, A.tile_cols(k)
        tt = kind == "tt"
        Td = self.TT if tt else self.TS
        ib = Td.mb
        kf = ents[0]["kf"]
        ld = max(e["ld"] for e in ents)
        wcols = sum(A.tile_cols(n) for n in cols)
        Vb, Tb = self.Vbs[k % len(self.Vbs)], self.Tbs[k % len(self.Tbs)]
        Yb = self.Ybs[k % len(self.Ybs)] if self.use_vt else None
        ygemm = GemmBatch() if self.use_vt else None
        gi, bi, panels, parts, ti = [], [], [], [], []
        for j, e in enumerate(ents):
            pb, vb, tb = j * ld * nb, vbase + j * ld * nb, tbase + j * nb * nb
            if e["direct"] is not None:
                ldp, rbl, rstride, poff = e["direct"]
                panels.append((A.data, poff, ldp, rbl, rstride, e["M"], kb, kf, Vb, vb, ld, Tb, tb, nb))
            else:
                g_ = e["gather"].items.copy()
                g_["b_off"] += pb
                b_ = e["back"].items.copy()
                b_["a_off"] += pb
                gi.append(g_)
                bi.append(b_)
                panels.append((self.Pb, pb, ld, 0, 0, e["M"], kb, kf, Vb, vb, ld, Tb, tb, nb))
            parts.append((e["rows"], vb + np.asarray(e["voff"], dtype=np.int64), j * kf * wcols, tb))
            if ygemm is not None:
                ygemm.add(vb, e["M"], kf, [(vb, tb, kf)])     # Y(entry) = V(entry) T(entry)^T
            row = e["rows"][1] if tt else e["rows"][0]
            for b0 in range(0, kf, ib):
                bs = min(ib, kf - b0)
                ti.append((tb + b0 * nb + b0, Td.offset(row, k) + b0 * Td.ld, bs, bs, 0, 0))
        def _tb(arrs):
            if not arrs:
                return None
            t = TileBatch()
            t.items = np.concatenate(arrs)
            t.max_m, t.max_n = int(t.items["m"].max()), int(t.items["n"].max())
            return t
        tst = TileBatch()
        for (a, b_, m_, n_, _, _) in ti:
            tst.add(a, m_, n_, b_off=b_)
        keep = torch.empty(len(ents) * kf * kf, dtype=A.dtype, device=A.device)
        store = getattr(Td, "full_T", None)
        if store is None:
            store = Td.full_T = {}
        for j, e in enumerate(ents):
            store[((e["rows"][1] if tt else e["rows"][0]), k)] = keep[j * kf * kf:(j + 1) * kf * kf]
        g = {"tt": tt, "n": len(ents), "ld": ld, "kf": kf, "zero": tt and bool(gi), "Vb": Vb, "Tb": Tb, "tb0": tbase,
             "plen": len(ents) * ld * nb, "gather": _tb(gi), "back": _tb(bi), "part": PART_UPPER if tt else PART_FULL,
             "multi": ops.QrPanelMulti(panels, A.dtype, A.device), "Td": Td, "tstore": tst.finalize(), "keep": keep,
             "Yb": Yb, "ygemm": ygemm.finalize() if ygemm is not None else None}
        if self.bla:
            g["next"] = _LeftMulti(A, [(r, v, j * kf * nb, t) for j, (r, v, _, t) in enumerate(parts)], kf,
                                   [n for n in cols if n == k + 1])
            g["rest"] = _LeftMulti(A, parts, kf, [n for n in cols if n != k + 1])
        else:
            g["upd"] = _LeftMulti(A, parts, kf, cols)
        return g

    def _panel_group(self, g):
        A = self.A
        nb = A.nb
        Tb = g["Tb"]
        # (a predicated step -- models/lu_qr.py -- still factors its panel: only scratch buffers are written
        # here, and the kernel must see a whole panel either way)
        with unpredicated():
            if g["zero"]:
                self.Pb[: g["plen"]].zero_()
            if g["gather"] is not None:
                ops.geadd(g["part"], N_, 1.0, A.data, A.ld, 0.0, self.Pb, g["ld"], g["gather"], copy=True)
            g["multi"].run(self.info)
        if g["back"] is not None:
            ops.geadd(g["part"], N_, 1.0, self.Pb, g["ld"], 0.0, A.data, A.ld, g["back"], copy=True)
        Td = g["Td"]
        ops.geadd(PART_FULL, N_, 1.0, Tb, nb, 0.0, Td.data, Td.ld, g["tstore"], copy=True)
        if g["ygemm"] is not None:
            ops.gemm(N_, T_, 1.0, g["Vb"], g["ld"], Tb, nb, 0.0, g["Yb"], g["ld"], g["ygemm"])
        n, kf, t0 = g["n"], g["kf"], g["tb0"]
        if kf == nb:
            g["keep"].view(n, kf * kf).copy_(Tb[t0: t0 + n * nb * nb].view(n, nb * nb))
        else:
            for j in range(n):
                torch.as_strided(g["keep"], (kf, kf), (1, kf), j * kf * kf).copy_(
                    torch.as_strided(Tb, (kf, kf), (1, nb), t0 + j * nb * nb))

    def step_batched(self, k):
        """One panel step in order (no look-ahead, or LU-QR's QR steps)."""
        if self.bla:
            self.panels_b(k)
            self.nexts_b(k)
            self.rests_b(k)
            return
        for g in self.bsteps[k]:
            self._panel_group(g)
            g["upd"].run(self.A, g["Vb"], g["ld"], g["Tb"], self.A.nb, self.Wb, self.W2b, qt=True, Yv=g["Yb"])

    # ---- batched look-ahead: panels of every group (TS launch, then each TT round) on the panel stream
    def panels_b(self, k):
        for g in self.bsteps[k]:
            self._panel_group(g)

    def nexts_b(self, k):
        for g in self.bsteps[k]:
            g["next"].run(self.A, g["Vb"], g["ld"], g["Tb"], self.A.nb, self.Wn, self.W2n, qt=True, Yv=g["Yb"])

    def rests_b(self, k):
        # DPLASMA_QR_REST_CAP=n: the bulk update as grid-stride GEMM launches of at most n workgroups, leaving
        # CUs to the next step's panel launches beside it (measurement knob; 0 = uncapped)
        cap = int(os.environ.get("DPLASMA_QR_REST_CAP", "0"))
        with (ops.gemm_wg_cap(cap) if cap > 0 else contextlib.nullcontext()):
            for g in self.bsteps[k]:
                g["rest"].run(self.A, g["Vb"], g["ld"], g["Tb"], self.A.nb, self.Wb, self.W2b, qt=True, Yv=g["Yb"])

    def _entry(self, k, rows, tt):
        A = self.A
        g = A.grid
        kb = A.tile_cols(k)
        voff, c = [], 0
        for r in rows:
            voff.append(c)
            c += A.tile_rows(r)
        M = c
        pc = g.pcol(k + A.jt0)
        rp = _prow(A, rows[0])
        rm = _prow(A, rows[1]) if tt else rp
        e = {"rows": rows, "voff": voff, "M": M, "kb": kb, "kf": min(M, kb), "tt": tt, "ld": max(16, _rup(M, 16)),
             "root": g.rank(rp, pc), "rp": rp, "rm": rm, "cross": rm != rp, "direct": None,
             "partner": g.rank(rm, pc)}
        # ranks of the reflector rows' process row(s) take part; the root factors
        e["own"] = A.rank == e["root"]
        e["is_partner"] = e["cross"] and A.rank == e["partner"]
        e["myline"] = A.myrow in (rp, rm)
        if e["cross"] and e["myline"]:
            other = rm if A.myrow == rp else rp
            e["peer"] = g.rank(other, A.mycol)      # the same process column in the other row
        if e["is_partner"]:
            m = rows[1]
            rb = TileBatch().add(A.offset(m, k), A.tile_rows(m), kb, b_off=0)
            e["r_out"] = rb.finalize()   # A(m,k) -> R buffer (ld = tile rows); upper part is R_m
            vb = TileBatch().add(voff[1], A.tile_rows(m), kb, b_off=A.offset(m, k))
            e["v_back"] = vb.finalize()  # V2 (upper) -> A(m,k)
        if not e["own"]:
            return e
        g_, back = TileBatch(), TileBatch()
        part = PART_UPPER if tt else PART_FULL
        for j, (r, o) in enumerate(zip(rows, voff)):
            if e["cross"] and j == 1:
                continue
            g_.add(A.offset(r, k), A.tile_rows(r), kb, b_off=o)
            back.add(o, A.tile_rows(r), kb, b_off=A.offset(r, k))
        e["gather"], e["back"], e["part"] = g_.finalize(), back.finalize(), part
        if e["cross"]:
            rin = TileBatch().add(0, A.tile_rows(rows[1]), kb, b_off=voff[1])
            e["r_in"] = rin.finalize()   # R buffer -> P (upper part)
        # a domain of consecutive tile rows stored contiguously is factored in place
        if not tt and self.inplace and list(rows) == list(range(rows[0], rows[0] + len(rows))) and g.P == 1:
            if A.storage == "tile" or A.ld == A.mb:
                e["direct"] = (A.mb, A.mb, A.mb * A.nb, A.offset(rows[0], k))
            else:
                e["direct"] = (A.ld, 0, 0, A.offset(rows[0], k))
        return e

    def _build(self, k):
        A = self.A
        doms, tts = self.plans[k]
        out = []
        cols = [n for n in range(k + 1, A.nt) if A.col_is_local(n)]
        nxt_c = [n for n in cols if n == k + 1]
        rest_c = [n for n in cols if n != k + 1]
        for d in doms:
            e = self._entry(k, d, False)
            if self.simple:
                e["next"] = _Left(A, d, e["voff"], e["kf"], nxt_c) if nxt_c else None
                e["rest"] = _Left(A, d, e["voff"], e["kf"], rest_c) if rest_c else None
            elif self.la:
                live = e["myline"]
                e["next"] = _Left(A, d, e["voff"], e["kf"], nxt_c) if (nxt_c and live) else None
                e["rest"] = _Left(A, d, e["voff"], e["kf"], rest_c) if (rest_c and live) else None
            else:
                e["upd"] = _Left(A, d, e["voff"], e["kf"], cols) if (cols and e["myline"]) else None
            out.append(e)
        for (p, ms) in tts:
            e = self._entry(k, [p] + list(ms), True)
            if e["cross"] and e["myline"]:   # only my process row's reflector row: partial W summed with the peer
                j = 0 if A.myrow == e["rp"] else 1
                rows, voff = [e["rows"][j]], [e["voff"][j]]
            else:
                rows, voff = e["rows"], e["voff"]
            if self.la:
                # a cross-row kill sums partial W with the peer: both rows must issue the exchange, so the
                # next / rest parts exist on both rows whenever the other one has columns there
                e["next"] = _Left(A, rows, voff, e["kf"], nxt_c) if (e["myline"] and nxt_c) else None
                e["rest"] = _Left(A, rows, voff, e["kf"], rest_c) if (e["myline"] and rest_c) else None
            else:
                e["upd"] = _Left(A, rows, voff, e["kf"], cols) if (cols and e["myline"]) else None
            out.append(e)
        return out

    def panel(self, k, e, buf, pbuf=None):
        """Assemble, factor, write back, store T of one domain / TT stack."""
        A = self.A
        P, V, Tm = self.P[buf if pbuf is None else pbuf], self.V[buf], self.Tm[buf]
        ld, M, kb, kf = e["ld"], e["M"], e["kb"], e["kf"]
        if e["is_partner"]:
            # cross-row TT, partner side: R_m to the root, V2 and T back, V2 into A(m,k)
            m = e["rows"][1]
            rows_m = A.tile_rows(m)
            ops.geadd(PART_FULL, N_, 1.0, A.data, A.ld, 0.0, self.R, rows_m, e["r_out"], copy=True)
            comm.p2p(sends=[(self.R[: rows_m * kb], e["root"])])
            comm.p2p(recvs=[(V[: ld * kf], e["root"]), (Tm, e["root"])])
            ops.geadd(PART_UPPER, N_, 1.0, V, ld, 0.0, A.data, A.ld, e["v_back"], copy=True)
            _store_T(Tm, A.nb, kf, self.TT, m, k)
            _keep_full_T(Tm, A.nb, kf, self.TT, m, k)
            self._bcast(e, V, Tm, e["partner"])
            return
        if not e["own"]:
            if e["myline"]:
                self._bcast(e, V, Tm, e["root"] if A.myrow == e["rp"] else e["partner"])
            return
        if e["direct"] is not None:
            ldp, rbl, rstride, poff = e["direct"]
            ops.qr_panel(A.data, ldp, M, kb, kf, V, ld, Tm, A.nb, self.ws, self.info, rbl=rbl, rstride=rstride,
                         poff=poff)
        else:
            if e["tt"]:
                P[: ld * kb].zero_()
            ops.geadd(e["part"], N_, 1.0, A.data, A.ld, 0.0, P, ld, e["gather"], copy=True)
            if e["cross"]:
                rows_m = A.tile_rows(e["rows"][1])
                comm.p2p(recvs=[(self.R[: rows_m * kb], e["partner"])])
                ops.geadd(PART_UPPER, N_, 1.0, self.R, rows_m, 0.0, P, ld, e["r_in"], copy=True)
            ops.qr_panel(P, ld, M, kb, kf, V, ld, Tm, A.nb, self.ws, self.info)
            ops.geadd(e["part"], N_, 1.0, P, ld, 0.0, A.data, A.ld, e["back"], copy=True)
        if e["cross"]:
            comm.p2p(sends=[(V[: ld * kf], e["partner"]), (Tm, e["partner"])])
        elif e["tt"]:
            _store_T(Tm, A.nb, kf, self.TT, e["rows"][1], k)
            _keep_full_T(Tm, A.nb, kf, self.TT, e["rows"][1], k)
        else:
            _store_T(Tm, A.nb, kf, self.TS, e["rows"][0], k)
            _keep_full_T(Tm, A.nb, kf, self.TS, e["rows"][0], k)
        self._bcast(e, V, Tm, e["root"])

    def _bcast(self, e, V, Tm, root):
        """V and T along my process row (from the rank of my row that holds them); T is upper
        triangular and only its triangle travels."""
        if self.vsend_task and self._cur_k is not None and self.A.rank == root:
            self._vq.setdefault(self._cur_k, []).append((e, V, Tm, root))
            return
        if self.dist and self.A.grid.Q > 1:
            comm.bcast(V[: e["ld"] * e["kf"]], root, self.ctx.row_group)
            nb = self.A.nb
            comm.bcast_tri(Tm, 0, Tm if self.A.rank == root else None, 0, e["kf"], nb, nb, False, root,
                           self.ctx.row_group)

    def apply(self, e, upd, buf, work, tmp=None):
        if upd is None:
            return
        red = None
        if e.get("cross"):
            t = self.xtmp if tmp is None else tmp
            red = lambda w, peer=e["peer"], t=t: comm.exchange_add(w, peer, t)  # noqa: E731
        upd.run(self.A, self.V[buf], e["ld"], self.Tm[buf], self.A.nb, *work, qt=True, reduce=red)

    # ---- general trees with look-ahead (self.la): V / T of entry i of step k in buffer (k % 2) * nent + i
    def panels_la(self, k):
        self._cur_k = k
        try:
            for i, e in enumerate(self.steps[k]):
                self.panel(k, e, (k % 2) * self.nent + i, pbuf=0)
        finally:
            self._cur_k = None

    def vsend(self, k):
        """The root broadcasts deferred by panels_la(k), in their order."""
        for e, V, Tm, root in self._vq.pop(k, []):
            self._bcast(e, V, Tm, root)

    def nexts_la(self, k):
        for i, e in enumerate(self.steps[k]):
            self.apply(e, e.get("next"), (k % 2) * self.nent + i, self.wn, self.xtmp_n)

    def rests_la(self, k):
        for i, e in enumerate(self.steps[k]):
            self.apply(e, e.get("rest"), (k % 2) * self.nent + i, self.wr, self.xtmp)

    def step_general(self, k):
        """One whole panel step in order (LU-QR's QR steps): look-ahead entries carry next / rest parts."""
        if self.la:
            self.panels_la(k)
            self.nexts_la(k)
            self.rests_la(k)
            return
        for e in self.steps[k]:
            self.panel(k, e, 0)
            self.apply(e, e.get("upd"), 0, self.wr)


def factor_New(ctx, A, TS, TT, tree, name="geqrf") -> Taskpool:
    """Build the taskpool of the stacked-domain QR (see module docstring)."""
    tp = Taskpool(name, ctx)
    tp.flops = flops(A.prec, "geqrf", A.m, A.n)
    TS.qr_format = TT.qr_format = "panel"
    st = _Factor(ctx, A, TS, TT, tree)
    if st.simple:
        prev_next = prev_rest = prev_rest2 = None
        for k in range(st.kt):
            e = st.steps[k][0]
            buf = k % 2
            pan = tp.task(f"qr_panel({k})", "panel", (lambda k=k, e=e, b=buf: st.panel(k, e, b)),
                          [prev_next, prev_rest2])
            nxt = None
            if e.get("next"):
                nxt = tp.task(f"qr_next({k})", "panel", (lambda e=e, b=buf: st.apply(e, e["next"], b, st.wn)),
                              [pan, prev_rest])
            rst = None
            if e.get("rest"):
                rst = tp.task(f"qr_rest({k})", "update", (lambda e=e, b=buf: st.apply(e, e["rest"], b, st.wr)),
                              [pan, prev_rest])
            prev_next, prev_rest2, prev_rest = nxt or pan, prev_rest, rst or prev_rest
    elif st.batched and st.bla:
        prev_next = prev_rest = prev_rest2 = None
        for k in range(st.kt):
            pan = tp.task(f"qr_panels({k})", "panel", (lambda k=k: st.panels_b(k)), [prev_next, prev_rest2])
            nxt = tp.task(f"qr_next({k})", "panel", (lambda k=k: st.nexts_b(k)), [pan, prev_rest])
            rst = tp.task(f"qr_rest({k})", "update", (lambda k=k: st.rests_b(k)), [pan, prev_rest])
            prev_next, prev_rest2, prev_rest = nxt, prev_rest, rst
    elif st.batched:
        prev = None
        for k in range(st.kt):
            prev = tp.task(f"qr_step({k})", "update", (lambda k=k: st.step_batched(k)), [prev])
    elif st.la:
        prev_next = prev_rest = prev_rest2 = None
        vs = {}
        for k in range(st.kt):
            # V / T buffers alternate with k's parity: step k+2's panels wait for step k's deferred broadcasts too
            pan = tp.task(f"qr_panel({k})", "panel", (lambda k=k: st.panels_la(k)), [prev_next, prev_rest2, vs.get(k - 2)])
            if st.vsend_task:
                vs[k] = tp.task(f"qr_vsend({k})", "vsend" if A.device.type == "cuda" else "update",
                                (lambda k=k: st.vsend(k)), [pan])
            nxt = tp.task(f"qr_next({k})", "panel", (lambda k=k: st.nexts_la(k)), [pan, prev_rest])
            rst = tp.task(f"qr_rest({k})", "update", (lambda k=k: st.rests_la(k)), [pan, prev_rest])
            prev_next, prev_rest2, prev_rest = nxt, prev_rest, rst
        if vs:
            tp.task("qr_vsend_join", "update", (lambda: None), [rst] + list(vs.values())[-2:])
    else:
        prev = None
        for k in range(st.kt):
            prev = tp.task(f"qr_step({k})", "update", (lambda k=k: st.step_general(k)), [prev])
    tp._state = st

    def _done():
        v = int(st.info.item())
        if v != 0:
            raise RuntimeError(f"QR panel kernel reported {v} (grid barrier timeout: is the device shared?)")
        return 0
    tp.on_complete(_done)
    return tp.finish_build()


# ----------------------------------------------------------------------------- applications
class _Apply:
    """C := op(Q) C or C op(Q) with Q in the stacked-domain format (unmqr / ungqr).

    P x Q grids: the reflectors of an item are built by the rank holding their storage (the domain
    owner; for a TT kill the owner of A(m,k), whose upper triangle is V2) and travel along the
    process row(s) of the reflector rows (left side; a cross-row TT also goes to the other row's
    panel-column rank, and the two rows sum their partial W pairwise) or to every rank (right side:
    the reflector rows are C's columns, the partial W is all-reduced along each process row)."""

    def __init__(self, ctx, side, trans, A, TS, TT, C, tree):
        self.ctx, self.A, self.TS, self.TT, self.C = ctx, A, TS, TT, C
        self.dist = ctx.world > 1
        self.pq = A.grid.P > 1
        dev, dt = A.device, A.dtype
        self.left = side == dplasmaLeft
        self.qt = trans in (dplasmaTrans, dplasmaConjTrans)
        if self.pq and self.left and (C.grid.P != A.grid.P or any(
                C.grid.prow(m + C.it0) != _prow(A, m) for m in range(min(C.mt, A.mt)))):
            raise ValueError("unmqr: C's tile rows must be distributed like A's")
        asc = (self.left and self.qt) or (not self.left and not self.qt)
        seq = _sequence(A, tree)
        self.seq = seq if asc else seq[::-1]
        self.ldv = max(16, _rup(A.m, 16))
        self.V = torch.zeros(self.ldv * A.nb, dtype=dt, device=dev)
        self.Tm = torch.zeros(A.nb * A.nb, dtype=dt, device=dev)
        self.items = [self._build(s) for s in self.seq]
        ups = [it["upd"] for it in self.items if it["upd"]]
        self.work = _work_buffers(ups, dt, dev)
        self.xtmp = torch.zeros(max([u.wlen for u in ups] + [1]), dtype=dt, device=dev)

    def _build(self, s):
        A, C = self.A, self.C
        g = A.grid
        k = s[1]
        tt = s[0] == "tt"
        rows = [s[2]] + list(s[3]) if tt else s[2]
        kb = A.tile_cols(k)
        voff, c = [], 0
        for r in rows:
            voff.append(c)
            c += A.tile_rows(r)
        M, kf = c, min(c, kb)
        pc = g.pcol(k + A.jt0)
        rp = _prow(A, rows[0])
        rm = _prow(A, rows[1]) if tt else rp
        holder = g.rank(rm, pc)
        it = {"k": k, "tt": tt, "rows": rows, "M": M, "kf": kf, "own": A.rank == holder, "root": holder,
              "rp": rp, "rm": rm, "cross": rm != rp, "relay": g.rank(rp, pc), "upd": None}
        mycols = [n for n in range(C.nt) if C.col_is_local(n)]
        if self.left:
            if not self.pq:
                it["upd"] = _Left(C, rows, voff, kf, mycols)
            elif C.myrow in (rp, rm) and mycols:
                if it["cross"]:
                    j = 0 if C.myrow == rp else 1
                    it["upd"] = _Left(C, [rows[j]], [voff[j]], kf, mycols)
                    it["peer"] = g.rank(rm if j == 0 else rp, C.mycol)
                else:
                    it["upd"] = _Left(C, rows, voff, kf, mycols)
        else:
            loc = [j for j, r in enumerate(rows) if C.col_is_local(r)]
            myrows = [i for i in range(C.mt) if C.row_is_local(i)]
            it["upd"] = _Right(C, myrows, [rows[j] for j in loc], [voff[j] for j in loc], kf,
                               split=not self.dist)
        if not it["own"]:
            return it
        # V gather batches: copy part (dom head: strictly lower / victims: full; TT: upper of m) + unit diagonal
        cp, dg = TileBatch(), TileBatch()
        if tt:
            dg.add(0, A.tile_rows(rows[0]), kf)
            for r, o in zip(rows[1:], voff[1:]):
                cp.add(A.offset(r, k), A.tile_rows(r), kf, b_off=o)
            it["cp"] = [(PART_UPPER, cp.finalize())]
        else:
            dg.add(0, A.tile_rows(rows[0]), kf)
            head, rest = TileBatch(), TileBatch()
            head.add(A.offset(rows[0], k), A.tile_rows(rows[0]), kf, b_off=0)
            for r, o in zip(rows[1:], voff[1:]):
                rest.add(A.offset(r, k), A.tile_rows(r), kf, b_off=o)
            it["cp"] = [(PART_SLOWER, head.finalize()), (PART_FULL, rest.finalize())]
        it["diag"] = dg.finalize()
        return it

    def _deliver(self, it, V, ld, kf):
        """V and T from the holder to every rank whose part of C they update."""
        A, ctx = self.A, self.ctx
        if not self.dist:
            return
        v = V[: ld * kf]
        nb = A.nb
        if not self.pq:                       # 1 x Q: along the (only) process row
            comm.bcast(v, it["root"], ctx.row_group)
            comm.bcast_tri(self.Tm, 0, self.Tm if A.rank == it["root"] else None, 0, kf, nb, nb, False,
                           it["root"], ctx.row_group)
            return
        if not self.left:                     # reflector rows = C's columns: every rank
            comm.bcast(v, it["root"], None, world=True)
            comm.bcast(self.Tm, it["root"], None, world=True)
            return
        if it["cross"]:                       # the other row's panel-column rank relays to its row
            if A.rank == it["root"]:
                comm.p2p(sends=[(v, it["relay"]), (self.Tm, it["relay"])])
            elif A.rank == it["relay"]:
                comm.p2p(recvs=[(v, it["root"]), (self.Tm, it["root"])])
        if A.myrow in (it["rp"], it["rm"]) and A.grid.Q > 1:
            src = it["root"] if A.myrow == it["rm"] else it["relay"]
            comm.bcast(v, src, ctx.row_group)
            comm.bcast_tri(self.Tm, 0, self.Tm if A.rank == src else None, 0, kf, nb, nb, False, src,
                           ctx.row_group)

    def run_item(self, it):
        A = self.A
        V, ld, kf = self.V, self.ldv, it["kf"]
        if it["own"]:
            V[: ld * kf].zero_()
            for part, b in it["cp"]:
                if len(b):
                    ops.geadd(part, N_, 1.0, A.data, A.ld, 0.0, V, ld, b, copy=True)
            ops.laset(PART_DIAG, 0.0, 1.0, V, ld, it["diag"])
            Td, row = (self.TT, it["rows"][1]) if it["tt"] else (self.TS, it["rows"][0])
            _rebuild_T(V, ld, it["M"], kf, Td, row, it["k"], self.Tm, A.nb)
        self._deliver(it, V, ld, kf)
        if it["upd"] is None:
            return
        red = None
        if self.left and it.get("peer") is not None:
            red = lambda w, peer=it["peer"]: comm.exchange_add(w, peer, self.xtmp)  # noqa: E731
        if self.left:
            it["upd"].run(self.C, V, ld, self.Tm, A.nb, *self.work, qt=self.qt, reduce=red)
        else:
            it["upd"].run(self.C, V, ld, self.Tm, A.nb, *self.work, qt=self.qt,
                          group=self.ctx.row_group if (self.dist and A.grid.Q > 1) else None)

    def run(self):
        for it in self.items:
            self.run_item(it)


def apply_New(ctx, side, trans, A, TS, TT, C, tree, name="unmqr") -> Taskpool:
    if C.dtype != A.dtype or (side == dplasmaLeft and C.mb != A.mb) or (side != dplasmaLeft and C.nb != A.mb):
        raise ValueError("C must share A's precision and tiling along the reflector dimension")
    tp = Taskpool(name, ctx)
    tp.flops = flops(A.prec, "unmqr", C.m, C.n, min(A.m, A.n), side == dplasmaLeft)
    st = _Apply(ctx, side, trans, A, TS, TT, C, tree)
    tp.task(name, "update", st.run, [])
    tp._state = st
    return tp.finish_build()
