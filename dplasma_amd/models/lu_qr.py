"""Hybrid LU-QR factorization (per panel: a stable-enough LU step, else an HQR step).

Reference: ``src/zgetrf_qrf.jdf`` (LU part: ``zgetrf`` / ``swptrsm_u`` /
``ztrsm_l`` / ``zgemm`` :77-276; QR part ``zgeqrt`` / ``zunmqr`` / ``zttqrt`` /
``zttmqr`` :277-640; decision: ``copypanel`` :645, ``zlufacto`` :739,
``reduce_norm`` :847, ``setchoice`` :937-1150, ``selector`` :1193),
``src/ztrsmpl_qrf.jdf``, ``src/zgetrf_qrf_wrapper.c`` (random LU table
``dplasma_genrandom_lutab``), ``src/include/dplasma/lu_qr.h`` (criteria) and
``tests/testing_zgetrf_qrf.c`` (trsmpl_qrf + trsm(U) solve check).

Semantics (as the reference): at step k the *diagonal domain* is the set of
panel tiles m = k, k+p, k+2p, ... (p = process-grid rows: the tiles that live
with the diagonal tile).  They are stacked and factored by LU with partial
pivoting; a criterion then compares a measure of that factorization with the
off-domain tiles of the panel:

=====================  =========================================================
DEFAULT (0)            alternate: LU on odd steps
HIGHAM (1)             alpha * cond(U_kk) > sum_i ||A_ik||_1
MUMPS (2)              alpha * max|A_kk(:,j)| >= max_i max|A_ik(:,j)| for all j
LU_ONLY / QR_ONLY      always LU / always QR
RANDOM (5)             lu_tab from a balanced random split with alpha % LU steps
HIGHAM_SUM/MAX/MOY     alpha / ||(L U)_kk^-1||_1 > sum / max / mean of ||A_ik||_1
=====================  =========================================================

alpha = 0 forces QR, alpha >= 9999999999 forces LU, a singular domain forces QR.
An LU step swaps rows inside the domain stack of every trailing column, solves
A(k, n) with L_kk, the off-domain A(m, k) with U_kk (no pivoting across
domains -- what the criterion guards) and updates the trailing matrix; a QR
step is one panel of hierarchical QR on the given tree.  lu_tab[k] records the
choice (1 = LU); IPIV(k, k) holds the domain pivots (1-based rows of the stack).

MI355X design: the domain LU runs on a contiguous copy of the stacked domain
tiles on the diagonal owner (the GPU panel kernel), so A's panel is untouched
until the decision -- the QR fallback needs no restore copy.  The decision is
one small allreduce (criterion values + pivots + info) per step; the LU step is
a TileProgram (row moves with the row-gather kernel, then batched TRSM and
MFMA GEMM launches) and the QR step a one-panel tile DAG (GEQRT / TTQRT /
TSMQR / TTMQR batched kernels, models/qr.py).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..constants import (dplasmaConjTrans, dplasmaLeft, dplasmaLower, dplasmaNoTrans, dplasmaNonUnit, dplasmaRight,
                         dplasmaUnit, dplasmaUpper)
from ..descriptor import TiledMatrix
from ..ops import qr_ops
from ..ops import tile_ops as ops
from ..ops.batch import GemmBatch, TileBatch
from ..ops.batch import unpredicated as ops_batch_unpredicated
from ..parallel import comm
from ..runtime.dag import TileDAG
from ..runtime.taskpool import Taskpool
from ..runtime.tileprog import TileProgram
from ..utils.flops import flops
from . import qr, qr_panel, qrtree
from .lu import _perm_from_swaps, _permute_rows_2d

DEFAULT_CRITERIUM = 0
HIGHAM_CRITERIUM = 1
MUMPS_CRITERIUM = 2
LU_ONLY_CRITERIUM = 3
QR_ONLY_CRITERIUM = 4
RANDOM_CRITERIUM = 5
HIGHAM_SUM_CRITERIUM = 6
HIGHAM_MAX_CRITERIUM = 7
HIGHAM_MOY_CRITERIUM = 8
_HIGHAMS = (HIGHAM_CRITERIUM, HIGHAM_SUM_CRITERIUM, HIGHAM_MAX_CRITERIUM, HIGHAM_MOY_CRITERIUM)

N_ = dplasmaNoTrans


def qrf_ipiv_descriptor(ctx, A, name="IPIV") -> TiledMatrix:
    """Pivot storage aligned with A: tile (k, k) (mb ints) holds step k's domain pivots."""
    return TiledMatrix(torch.int32, A.mb, 1, A.mt * A.mb, A.nt, P=A.grid.P, Q=A.grid.Q, rank=A.rank,
                       device=A.device, name=name)


def genrandom_lutab(lu_tab, deb, fin, nb_lu, rec_depth=0):
    """Balanced recursive split of nb_lu LU steps over [deb, fin] (dplasma_genrandom_lutab)."""
    if deb == fin:
        lu_tab[deb] = int(nb_lu != 0)
        return
    n = fin - deb + 1
    new_fin = deb - 1 + n // 2 if n % 2 == 0 else deb - 1 + (fin - deb) // 2 + (rec_depth % 2)
    new_nb = nb_lu // 2 if nb_lu % 2 == 0 else (nb_lu - 1) // 2 + (rec_depth % 2)
    genrandom_lutab(lu_tab, deb, new_fin, new_nb, rec_depth + 1)
    genrandom_lutab(lu_tab, new_fin + 1, fin, nb_lu - new_nb, rec_depth + 1)


def _w0(lu: torch.Tensor, crit: int) -> torch.Tensor:
    """The criterion's measure of the domain's square LU (a 0-d tensor on lu's device, no host sync):
    HIGHAM: cond_1(U) = ||U||_1 ||U^-1||_1; HIGHAM_SUM / MAX / MOY: 1 / ||(L U)^-1||_1.  Exact norms from
    the triangular inverses (the reference estimates them with LAPACK's trcon / gecon,
    src/zgetrf_qrf.jdf:739-846 -- the same quantities; a decision exactly at the estimate's error margin is
    parity unpinned)."""
    n = lu.shape[0]
    eye = torch.eye(n, dtype=lu.dtype, device=lu.device)
    U = torch.triu(lu)
    if crit == HIGHAM_CRITERIUM:
        Ui = torch.linalg.solve_triangular(U, eye, upper=True)
        return U.abs().sum(0).max() * Ui.abs().sum(0).max()
    L = torch.tril(lu, -1) + eye
    X = torch.linalg.solve_triangular(L, eye, upper=False, unitriangular=True)
    X = torch.linalg.solve_triangular(U, X, upper=True)
    return 1.0 / X.abs().sum(0).max()


class _Step:
    """Shared per-step geometry."""

    def __init__(self, A, k, p):
        self.k = k
        self.dom = list(range(k, A.mt, p))
        self.off = [m for m in range(k + 1, A.mt) if (m - k) % p]
        self.rows = [A.tile_rows(m) for m in self.dom]
        self.M = sum(self.rows)
        self.ncol = A.tile_cols(k)
        self.kmax = min(self.M, self.ncol)
        self.owner = A.rank_of(k, k)
        # global element rows of the stacked domain, in stack order
        self.grow = np.concatenate([np.arange(m * A.mb, m * A.mb + r) for m, r in zip(self.dom, self.rows)])


class _GetrfQrf(Taskpool):
    def __init__(self, ctx, tree, A, IPIV, TS, TT, criteria, alpha, lu_tab, info, p):
        super().__init__("getrf_qrf", ctx)
        self.tree, self.A, self.IPIV, self.TS, self.TT = tree, A, IPIV, TS, TT
        self.criteria, self.alpha = criteria, float(alpha)
        self.minMNT = min(A.mt, A.nt)
        self.lu_tab = lu_tab if lu_tab is not None else [0] * self.minMNT
        self.info_out = info
        self.p = p or A.grid.P
        self.kd = qr_ops.kinds(A.dtype, TS.mb, (0, 0), (0, 0))
        self._panel_ws = {}
        self._lu_batches = {}
        self._plu, self._pbuf = {}, None
        # QR steps on the stacked-domain engine (models/qr_panel.py: every TS domain of the step's tree
        # one persistent panel launch, TT kills likewise, MFMA trailing updates) when it handles A and the
        # tree; T factors then live in its ("panel") format and trsmpl_qrf applies them the same way
        self.qpf = None
        if qr_panel.usable(A, tree):
            # a data-dependent criterion may run device-decided (below): its QR panels then run under a predicate
            # they do not see, so none may factor in place in A
            maybe_dev = (((ctx.world == 1 and A.device.type == "cuda") or
                          (ctx.world > 1 and (p or A.grid.P) % A.grid.P == 0))
                         and (criteria in _HIGHAMS or criteria == MUMPS_CRITERIUM)
                         and os.environ.get("DPLASMA_LUQR_DEVCRIT", "1") != "0")
            self.qpf = qr_panel._Factor(ctx, A, TS, TT, tree, inplace=not maybe_dev)
            TS.qr_format = TT.qr_format = "panel"
        else:
            TS.qr_format = TT.qr_format = "tile"
        self.flops = flops(A.prec, "getrf", A.m, A.n)
        if criteria == RANDOM_CRITERIUM:
            genrandom_lutab(self.lu_tab, 0, self.minMNT - 1, int(round(self.minMNT * self.alpha / 100.0)), 0)
        # Device-resident path (one process, domain = the whole panel column, a criterion that does not
        # read the matrix): every step is issued without a host synchronisation -- LU steps on the
        # partial-pivoting engine of getrf_1d (models/lu.py _GetrfDev: device pivot search, device row
        # moves, MFMA updates; interchanges restricted to the trailing columns), QR steps on the
        # stacked-domain engine -- and no LU is factored for a step that will be QR.  An exactly singular
        # diagonal domain is reported through info at completion instead of turning that step into QR
        # (DPLASMA_LUQR_SYNC=1 keeps the reference's per-step host decision).
        self.fast = None
        # Device-decided steps (one GPU process, a criterion that reads the matrix, p > 1): every step's domain
        # LU, criterion and decision stay on the device and BOTH branches are issued predicated on the decision
        # flag (ops/batch.py predicated: the untaken branch's batched launches run with empty items) -- no
        # host synchronisation in the step loop; lu_tab is read back once at completion.
        # DPLASMA_LUQR_DEVCRIT=0 keeps the per-step host decision.
        self.devcrit = (ctx.world == 1 and A.device.type == "cuda" and self.qpf is not None and self.qpf.batched
                        and (criteria in _HIGHAMS or criteria == MUMPS_CRITERIUM) and self.alpha != 0
                        and self.alpha < 9999999999 and os.environ.get("DPLASMA_LUQR_DEVCRIT", "1") != "0"
                        and os.environ.get("DPLASMA_LUQR_SYNC", "0") != "1")
        # Several processes (the reference reduces the criterion inside the DAG: zlufacto -> reduce_norm ->
        # setchoice, src/zgetrf_qrf.jdf:739-1156): the diagonal owner's domain LU, w0 and pivots, every rank's
        # off-domain norms, the cross-rank reduction (device all-reduce: RCCL on GPUs) and the decision flag stay
        # on the device, and both branches are issued under the flag -- the LU branch's interchanges from a
        # device move list (the domain lives on one process row when p is a multiple of P), its solves and
        # update as a predicated tile program; the QR branch on the stacked-domain engine (no in-place panels).
        # On the CPU the batched fallbacks loop over host records and cannot see a predicate: there the flag is
        # read (no device to synchronise) and only the taken branch runs.
        self.devcrit_dist = (ctx.world > 1 and self.qpf is not None and not self.qpf.inplace
                             and (criteria in _HIGHAMS or criteria == MUMPS_CRITERIUM) and self.alpha != 0
                             and self.alpha < 9999999999 and self.p % A.grid.P == 0
                             and os.environ.get("DPLASMA_LUQR_DEVCRIT", "1") != "0"
                             and os.environ.get("DPLASMA_LUQR_SYNC", "0") != "1")
        self._dec = []
        if self.devcrit:
            # every step's tables, panel plans and workspaces now: the run issues no host round trip at all
            for k in range(self.minMNT):
                st = _Step(A, k, self.p)
                self._dev_step(st)
                key = (st.M, st.ncol)
                if key not in self._panel_ws:
                    self._panel_ws[key] = (ops.lu_workspace(st.M, A.device),
                                           torch.zeros(1, dtype=torch.int32, device=A.device))
        fast_env = os.environ.get("DPLASMA_LUQR_FAST", "auto")   # auto: on GPU; 1: also on CPU; 0: never
        if (ctx.world == 1 and self.p == 1 and fast_env != "0" and (A.device.type == "cuda" or fast_env == "1")
                and self._a_priori(0) is not None and os.environ.get("DPLASMA_LUQR_SYNC", "0") != "1"):
            from .lu import _GetrfDev
            self.fast_info = torch.zeros(1, dtype=torch.int32, device=A.device)
            la = os.environ.get("DPLASMA_LUQR_LOOKAHEAD", "1") != "0"
            # look-ahead issues PANEL(k+1) beside REST(k): the LU engine alternates its panel buffers
            # 32-column pivoting blocks beside the updates: 21.3-21.6 vs 20.5-20.7 TF/s at 32k (r4_b22, r4_b25)
            self.fast = _GetrfDev(ctx, A, self.fast_info, pivot=True, trailing_only=True, lookahead=la,
                                  panel_bw=32 if la else None)
            if la:
                self._fast_tasks()
        self.finish_build()

    def _fast_tasks(self):
        """Look-ahead across LU and QR steps (device path): every step is PANEL / NEXT on the panel
        stream and the bulk REST on the update stream, so step k+1's panel -- a pivoting LU panel or the
        QR step's TS + TT launches -- runs beside step k's trailing update.  LU: PANEL(k) -> SWAP(k)
        (after REST(k-1): the interchanges touch every trailing column) -> NEXT(k) || REST(k);
        QR: PANELS(k) -> NEXT(k) (after REST(k-1)) || REST(k) (V / T double-buffered by step parity)."""
        f, dev = self.qpf, self.fast
        if f is None or not (f.simple or (f.batched and f.bla)):
            return
        prev_next = prev_rest = None
        for k in range(self.minMNT):
            cond = self._a_priori(k)
            self.lu_tab[k] = cond
            if cond:
                pn = self.task(f"LU_PANEL({k})", "panel", (lambda k=k: self._lu_panel_fast(k)), [prev_next], prio=3)
                sw = self.task(f"LU_SWAP({k})", "update", (lambda k=k: dev.swap(k)), [pn, prev_rest], prio=2)
                prev_next = self.task(f"LU_NEXT({k})", "panel", (lambda k=k: dev.next(k)), [sw], prio=2)
                prev_rest = self.task(f"LU_REST({k})", "update", (lambda k=k: dev.rest(k)), [sw], prio=1)
            else:
                pn = self.task(f"QR_PANELS({k})", "panel", (lambda k=k: self._qr_panels_fast(k)), [prev_next], prio=3)
                nx = self.task(f"QR_NEXT({k})", "panel", (lambda k=k: self._qr_part_fast(k, "next")),
                               [pn, prev_rest], prio=2)
                prev_rest = self.task(f"QR_REST({k})", "update", (lambda k=k: self._qr_part_fast(k, "rest")),
                                      [pn, prev_rest], prio=1)
                prev_next = nx

    def _lu_panel_fast(self, k):
        dev = self.fast
        dev.panel(k)
        if self.IPIV.is_local(k, k):
            kmin = dev.plan[k]["kmin"]
            t = self.IPIV.tile(k, k)
            t.zero_()
            t[:kmin, 0] = dev.piv_dev[:kmin] + 1

    def _qr_panels_fast(self, k):
        f = self.qpf
        if self.IPIV.is_local(k, k):
            self.IPIV.tile(k, k).zero_()
        if f.simple:
            f.panel(k, f.steps[k][0], k % 2)
        else:
            f.panels_b(k)

    def _qr_part_fast(self, k, part):
        f = self.qpf
        if f.simple:
            e = f.steps[k][0]
            f.apply(e, e.get(part), k % 2, f.wn if part == "next" else f.wr)
        elif part == "next":
            f.nexts_b(k)
        else:
            f.rests_b(k)

    def _a_priori(self, k):
        """The step's choice when it does not depend on the data (1 LU, 0 QR), else None."""
        if self.alpha == 0:
            return 0
        if self.alpha >= 9999999999:
            return 1
        c = self.criteria
        if c == LU_ONLY_CRITERIUM:
            return 1
        if c == QR_ONLY_CRITERIUM:
            return 0
        if c == RANDOM_CRITERIUM:
            return int(self.lu_tab[k])
        if c in _HIGHAMS or c == MUMPS_CRITERIUM:
            if self.p != 1:
                return None
            # p = 1: the domain is the whole panel column, so no tile is off-domain: the off-domain
            # sum / max / column maxima are 0 and the decision does not depend on the data --
            # alpha * w0 > 0 (w0 > 0 for a non-singular domain), alpha * colmax >= 0; the mean over zero
            # off-domain tiles is 0 / 0 in the reference (src/zgetrf_qrf.jdf:1125-1135), NaN: never LU
            if c == HIGHAM_MOY_CRITERIUM:
                return 0
            if c == MUMPS_CRITERIUM:
                return 1 if self.alpha >= 0 else None
            return 1 if self.alpha > 0 else None
        return k % 2

    def _run_fast(self):
        A, dev = self.A, self.fast
        for k in range(self.minMNT):
            cond = self._a_priori(k)
            self.lu_tab[k] = cond
            if cond:
                dev.step(k)
                kmin = dev.plan[k]["kmin"]
                if self.IPIV.is_local(k, k):
                    t = self.IPIV.tile(k, k)
                    t.zero_()
                    t[:kmin, 0] = dev.piv_dev[:kmin] + 1
            else:
                self._qr_step(_Step(A, k, self.p))

    # ------------------------------------------------------------------ device-decided steps
    def _run_devcrit(self):
        from ..ops import batch as B
        A = self.A
        self._dec = []
        for k in range(self.minMNT):
            st = _Step(A, k, self.p)
            buf, view, ipiv, info, colmax = self._domain_lu_dev(st)
            flag = self._criterion_dev(st, view, info, colmax)
            self._dec.append(flag)
            with B.predicated(flag):
                self._lu_step_dev(st, buf, ipiv, flag)
            with B.predicated(1 - flag):
                self._qr_step(st, zero_ipiv=False)   # (the LU branch wrote IPIV(k, k) = flag * pivots)

    def _domain_lu_dev(self, st: _Step):
        """The stacked domain's LU on the device (a copy: A is untouched until the decision)."""
        A = self.A
        if self._pbuf is None:
            self._pbuf = torch.empty(max(1, A.m * A.nb), dtype=A.dtype, device=A.device)
        buf = self._pbuf[: st.ncol * st.M]
        view = torch.as_strided(buf, (st.M, st.ncol), (1, st.M))
        dv = self._dev_step(st)
        ops.geadd(0, N_, 1.0, A.data, A.ld, 0.0, buf, st.M, dv["gather"], copy=True)
        colmax = None
        if self.criteria == MUMPS_CRITERIUM:
            colmax = A.tile(st.k, st.k)[:st.ncol, :st.ncol].abs().amax(0)
        ipiv = torch.zeros(max(st.kmax, 1), dtype=torch.int32, device=A.device)
        info = torch.zeros(1, dtype=torch.int32, device=A.device)
        key = (st.M, st.ncol)
        ws = self._panel_ws.get(key)
        if ws is None:
            ws = self._panel_ws[key] = (ops.lu_workspace(st.M, A.device),
                                        torch.zeros(1, dtype=torch.int32, device=A.device))
        plu = self._plu.get(st.k)
        if plu is None:
            plu = self._plu[st.k] = ops.PanelLU(buf, st.M, st.M, st.ncol, pivot=True)
        plu.run(ipiv, ws[0], ws[1], info, 0)
        return buf, view, ipiv, info, colmax

    def _criterion_dev(self, st: _Step, view, info, colmax):
        """The step's decision as a device int32 flag [1] (1 = LU): _decide's formulas on device tensors."""
        A, crit, alpha = self.A, self.criteria, self.alpha
        bad = info[0] != 0
        offs = [A.tile(m, st.k) for m in st.off]
        if crit == MUMPS_CRITERIUM:
            if offs:
                off = torch.stack([t.abs().amax(0) for t in offs]).amax(0)[:st.ncol]
                cond = (alpha * colmax >= off).all()
            else:
                cond = torch.ones((), dtype=torch.bool, device=A.device)
        else:
            lu = view[:st.ncol, :st.ncol]
            w0 = torch.nan_to_num(_w0(lu, crit).to(torch.float64), nan=0.0, posinf=float("inf"))
            n1 = torch.stack([t.abs().sum(0).max() for t in offs]).to(torch.float64) if offs else None
            if crit in (HIGHAM_CRITERIUM, HIGHAM_SUM_CRITERIUM):
                thr = n1.sum() if offs else torch.zeros((), dtype=torch.float64, device=A.device)
                cond = alpha * w0 > thr
            elif crit == HIGHAM_MAX_CRITERIUM:
                thr = n1.max() if offs else torch.zeros((), dtype=torch.float64, device=A.device)
                cond = alpha * w0 > thr
            else:
                nt_ = A.mt - st.k
                nout = nt_ - (nt_ + self.p - 1) // self.p
                if nout == 0:
                    cond = torch.zeros((), dtype=torch.bool, device=A.device)   # 0 / 0: the reference's NaN
                else:
                    cond = alpha * w0 > n1.sum() / nout
        return (cond & ~bad).to(torch.int32).view(1)

    def _dev_step(self, st: _Step):
        """Per-step batches of the device-decided path (built once, cached): domain gather / write-back and the
        stacked-row table of the trailing row interchanges."""
        d = self.__dict__.setdefault("_devb", {}).get(st.k)
        if d is not None:
            return d
        A, k = self.A, st.k
        d = {}
        if A.rank == st.owner:   # the domain's tiles (all of column k's domain rows live with the diagonal tile)
            g, back = TileBatch(), TileBatch()
            r0 = 0
            for m, r in zip(st.dom, st.rows):
                g.add(A.offset(m, k), r, st.ncol, b_off=r0)
                back.add(r0, r, st.ncol, b_off=A.offset(m, k))
                r0 += r
            d["gather"], d["back"] = g.finalize(), back.finalize()
        # the trailing interchanges: my local trailing columns, when the domain rows are on my process row
        trail = [n for n in range(k + 1, A.nt) if A.col_is_local(n)] if A.row_is_local(k) else []
        if trail:
            base = A.offset(st.dom[0], trail[0])
            d["rowoff"] = torch.tensor([A.offset(m, trail[0]) - base for m in st.dom], dtype=torch.int64,
                                       device=A.device)
            d["coloff"] = torch.tensor([A.offset(st.dom[0], n) for n in trail], dtype=torch.int64, device=A.device)
            d["ncols"] = torch.tensor([A.tile_cols(n) for n in trail], dtype=torch.int32, device=A.device)
            nb = A.nb
            d["mv"] = (torch.zeros(2 * nb, dtype=torch.int32, device=A.device),
                       torch.zeros(2 * nb, dtype=torch.int32, device=A.device),
                       torch.zeros(1, dtype=torch.int32, device=A.device))
        self._devb[k] = d
        return d

    def _lu_step_dev(self, st: _Step, buf, ipiv, flag):
        """The LU branch, issued under the step's predicate: factored domain back into A, the pivots into IPIV,
        the interchanges inside the domain stack of every trailing column (device move list, its count
        multiplied by the flag), then the solves and the update (batched: predicated)."""
        A, k = self.A, st.k
        d = self._dev_step(st)
        ops.geadd(0, N_, 1.0, buf, st.M, 0.0, A.data, A.ld, d["back"], copy=True)
        if self.IPIV.is_local(k, k):
            t = self.IPIV.tile(k, k)
            new = torch.zeros_like(t)
            new[:st.kmax, 0] = ipiv[:st.kmax] + 1
            t.copy_(new * flag.to(t.dtype))
        if "rowoff" in d:
            mdst, msrc, mcnt = d["mv"]
            with ops_batch_unpredicated():
                ops.piv_moves(ipiv, st.kmax, mdst, msrc, mcnt, mrel=st.M, info=self._devinfo())
            mcnt.mul_(flag)
            ops.rows_permute(A.data, A.ld, A.mb, 0, d["rowoff"], d["coloff"], d["ncols"], A.nb, mdst, msrc, mcnt,
                             2 * A.nb, self._devinfo())
        self._lu_update_local(st)

    def _devinfo(self):
        t = self.__dict__.get("_dinfo")
        if t is None:
            t = self._dinfo = torch.zeros(1, dtype=torch.int32, device=self.A.device)
        return t

    # ------------------------------------------------------------------ device-decided steps, several processes
    def _run_devcrit_dist(self):
        from ..ops import batch as B
        A, ctx = self.A, self.ctx
        gpu = A.device.type == "cuda"
        self._dec = []
        for k in range(self.minMNT):
            st = _Step(A, k, self.p)
            mine = self._domain_lu_dev(st) if ctx.rank == st.owner else None
            flag, ipiv = self._decide_dev(st, mine)
            self._dec.append(flag)
            if gpu:
                with B.predicated(flag):
                    self._lu_step_dist_dev(st, mine, ipiv, flag)
                with B.predicated(1 - flag):
                    self._qr_step(st, zero_ipiv=False)   # (the LU branch wrote IPIV(k, k) = flag * pivots)
            elif int(flag[0]):
                self._lu_step_dist_dev(st, mine, ipiv, flag)
            else:
                self._qr_step(st)

    def _decide_dev(self, st: _Step, mine):
        """_decide on the device: the SUM vector [w0, bad, offsum, ipiv(nb), colmax_diag(nb)] and the MAX vector
        [offmax, colmax_off(nb)] filled by device ops, all-reduced on the device, the flag computed from them.
        Returns (flag int32 [1], pivots int32 [kmax]) -- the same on every rank, nothing read by the host."""
        A, crit, alpha = self.A, self.criteria, self.alpha
        dev, nb, k = A.device, A.nb, st.k
        f64 = torch.float64
        vs = torch.zeros(3 + 2 * nb, dtype=f64, device=dev)
        vm = torch.zeros(1 + nb, dtype=f64, device=dev)
        if mine is not None:
            _, view, ipiv, info, colmax = mine
            bad = info[0] != 0
            vs[1] = bad.to(f64)
            if crit in _HIGHAMS:
                w0 = torch.nan_to_num(_w0(view[:st.ncol, :st.ncol], crit).to(f64), nan=0.0, posinf=float("inf"))
                vs[0] = torch.where(bad, torch.zeros((), dtype=f64, device=dev), w0)
            vs[3:3 + st.kmax] = ipiv[:st.kmax].to(f64)
            if colmax is not None:
                vs[3 + nb:3 + nb + colmax.numel()] = colmax.to(f64)
        offs = [A.tile(m, k) for m in st.off if A.is_local(m, k)]
        if offs:
            if crit == MUMPS_CRITERIUM:
                cm = torch.stack([t.abs().amax(0) for t in offs]).amax(0).to(f64)
                vm[1:1 + cm.numel()] = cm
            else:
                n1 = torch.stack([t.abs().sum(0).max() for t in offs]).to(f64)
                vs[2] = n1.sum()
                vm[0] = n1.max()
        comm.allreduce(vs)
        comm.allreduce(vm, op=torch.distributed.ReduceOp.MAX)
        w0, offsum, offmax = vs[0], vs[2], vm[0]
        bad = vs[1] > 0
        if crit in (HIGHAM_CRITERIUM, HIGHAM_SUM_CRITERIUM):
            cond = alpha * w0 > offsum
        elif crit == HIGHAM_MAX_CRITERIUM:
            cond = alpha * w0 > offmax
        elif crit == HIGHAM_MOY_CRITERIUM:
            nt_ = A.mt - k
            nout = nt_ - (nt_ + self.p - 1) // self.p
            cond = (alpha * w0 > offsum / nout) if nout else torch.zeros((), dtype=torch.bool, device=dev)
        else:   # MUMPS
            cond = (alpha * vs[3 + nb:3 + nb + st.ncol] >= vm[1:1 + st.ncol]).all()
        flag = (cond & ~bad).to(torch.int32).view(1)
        return flag, vs[3:3 + st.kmax].round().to(torch.int32)

    def _lu_step_dist_dev(self, st: _Step, mine, ipiv, flag):
        """The LU branch on a P x Q grid, issued under the step's predicate: the owner writes the factored domain
        back, IPIV(k, k) = flag x pivots, the domain's process row permutes its local trailing columns from the
        device move list (count multiplied by the flag), then the solves and the update (tile program: batched
        launches, predicated; its operand transfers run whatever the flag -- they only read)."""
        A, k = self.A, st.k
        d = self._dev_step(st)
        if mine is not None:
            ops.geadd(0, N_, 1.0, mine[0], st.M, 0.0, A.data, A.ld, d["back"], copy=True)
        if self.IPIV.is_local(k, k):
            t = self.IPIV.tile(k, k)
            new = torch.zeros_like(t)
            new[:st.kmax, 0] = ipiv[:st.kmax] + 1
            t.copy_(new * flag.to(t.dtype))
        if "rowoff" in d:
            mdst, msrc, mcnt = d["mv"]
            with ops_batch_unpredicated():
                ops.piv_moves(ipiv, st.kmax, mdst, msrc, mcnt, mrel=st.M, info=self._devinfo())
            mcnt.mul_(flag)
            ops.rows_permute(A.data, A.ld, A.mb, 0, d["rowoff"], d["coloff"], d["ncols"], A.nb, mdst, msrc, mcnt,
                             2 * A.nb, self._devinfo())
        self._lu_update_prog(st)

    def _lu_update_prog(self, st: _Step):
        """The LU step's solves and trailing update on a P x Q grid (one tile program)."""
        A, ctx, k = self.A, self.ctx, st.k
        prog = TileProgram(ctx, f"getrf_qrf_lu({k})")
        s = prog.stage("trsm")
        for n in range(k + 1, A.nt):
            s.trsm(dplasmaLeft, dplasmaLower, N_, dplasmaUnit, 1.0, (A, k, k), (A, k, n))
        for m in st.off:
            s.trsm(dplasmaRight, dplasmaUpper, N_, dplasmaNonUnit, 1.0, (A, k, k), (A, m, k))
        if k + 1 < A.nt:
            s = prog.stage("gemm")
            for m in range(k + 1, A.mt):
                for n in range(k + 1, A.nt):
                    s.gemm((A, m, n), [((A, m, k), N_, (A, k, n), N_)], alpha=-1.0, beta=1.0)
        prog.compile().execute(ctx)

    # ------------------------------------------------------------------ one panel
    def _domain_lu(self, st: _Step):
        """Stacked LU of the domain on the diagonal owner -> (buffer, ipiv, info, W0, colmax)."""
        A = self.A
        if self._pbuf is None:
            self._pbuf = torch.empty(max(1, A.m * A.nb), dtype=A.dtype, device=A.device)
        buf = self._pbuf[: st.ncol * st.M]
        view = torch.as_strided(buf, (st.M, st.ncol), (1, st.M))
        r0 = 0
        for m, r in zip(st.dom, st.rows):
            view[r0:r0 + r].copy_(A.tile(m, st.k))
            r0 += r
        colmax = None
        if self.criteria == MUMPS_CRITERIUM:
            colmax = A.tile(st.k, st.k)[:st.ncol, :st.ncol].abs().amax(0).double().cpu().numpy()
        ipiv = torch.zeros(max(st.kmax, 1), dtype=torch.int32, device=A.device)
        info = torch.zeros(1, dtype=torch.int32, device=A.device)
        if A.device.type == "cuda":
            # the recursive device panel (persistent pivoting block kernels, TRSM / MFMA GEMM joins) --
            # the same engine as getrf_1d's PANEL task, not a one-workgroup panel
            key = (st.M, st.ncol)
            ws = self._panel_ws.get(key)
            if ws is None:
                ws = self._panel_ws[key] = (ops.lu_workspace(st.M, A.device),
                                            torch.zeros(1, dtype=torch.int32, device=A.device))
            plu = self._plu.get(st.k)
            if plu is None:
                plu = self._plu[st.k] = ops.PanelLU(buf, st.M, st.M, st.ncol, pivot=True)
            plu.run(ipiv, ws[0], ws[1], info, 0)
        else:
            ops.getrf_panel(buf, 0, st.M, st.ncol, st.M, ipiv, info, 0, pivot=True)
        w0 = 0.0
        bad = int(info.item()) != 0
        if not bad and self.criteria in _HIGHAMS:
            lu = view[:st.ncol, :st.ncol].cpu().to(torch.complex128 if A.dtype.is_complex else torch.float64)
            w0 = float(_w0(lu, self.criteria))
        return buf, view, ipiv, bad, w0, colmax

    def _offdomain_norms(self, st: _Step):
        """Local partial (sum, max, count) of off-domain tile 1-norms, or per-column max (MUMPS)."""
        A = self.A
        s, mx, cnt = 0.0, 0.0, 0
        cm = np.zeros(A.nb)
        for m in st.off:
            if not A.is_local(m, st.k):
                continue
            t = A.tile(m, st.k)
            if self.criteria == MUMPS_CRITERIUM:
                c = t.abs().amax(0).double().cpu().numpy()
                cm[:len(c)] = np.maximum(cm[:len(c)], c)
            else:
                v = float(t.abs().sum(0).max())
                s, mx, cnt = s + v, max(mx, v), cnt + 1
        return s, mx, cm

    def _decide(self, st: _Step, mine):
        """Collective decision: every rank returns the same (do_lu, ipiv)."""
        A, ctx = self.A, self.ctx
        me = ctx.rank
        s, mx, cm = self._offdomain_norms(st)
        nb = A.nb
        # SUM vector: [w0, bad, offsum, ipiv(nb), colmax_diag(nb)]; MAX vector: [offmax, colmax_off(nb)]
        vs = torch.zeros(3 + 2 * nb, dtype=torch.float64)
        vm = torch.zeros(1 + nb, dtype=torch.float64)
        if me == st.owner:
            _, _, ipiv, bad, w0, colmax = mine
            vs[0], vs[1] = (0.0 if bad else w0), float(bad)
            vs[3:3 + st.kmax] = ipiv[:st.kmax].double().cpu()
            if colmax is not None:
                vs[3 + nb:3 + nb + len(colmax)] = torch.from_numpy(colmax)
        vs[2] = s
        vm[0] = mx
        vm[1:] = torch.from_numpy(cm)
        if ctx.world > 1:
            dv = ctx.device
            a, b = vs.to(dv), vm.to(dv)
            comm.allreduce(a)
            comm.allreduce(b, op=torch.distributed.ReduceOp.MAX)
            vs, vm = a.cpu(), b.cpu()
        w0, bad, offsum, offmax = float(vs[0]), vs[1] > 0, float(vs[2]), float(vm[0])
        ipiv = vs[3:3 + st.kmax].round().to(torch.int64).numpy()
        k, alpha, crit = st.k, self.alpha, self.criteria
        if bad:
            cond = 0
        elif crit in (HIGHAM_CRITERIUM, HIGHAM_SUM_CRITERIUM):
            cond = int(alpha * w0 > offsum)
        elif crit == HIGHAM_MAX_CRITERIUM:
            cond = int(alpha * w0 > offmax)
        elif crit == HIGHAM_MOY_CRITERIUM:
            nt_ = A.mt - k
            nout = nt_ - (nt_ + self.p - 1) // self.p
            cond = int(alpha * w0 > (offsum / nout if nout else float("nan")))   # 0 / 0: the reference's NaN
        elif crit == MUMPS_CRITERIUM:
            diag = vs[3 + nb:3 + nb + st.ncol].numpy()
            off = vm[1:1 + st.ncol].numpy()
            cond = int(bool(np.all(alpha * diag >= off)))
        elif crit == LU_ONLY_CRITERIUM:
            cond = 1
        elif crit == QR_ONLY_CRITERIUM:
            cond = 0
        elif crit == RANDOM_CRITERIUM:
            cond = int(self.lu_tab[k])
        else:
            cond = k % 2
        if not bad:
            if alpha == 0:
                cond = 0
            if alpha >= 9999999999:
                cond = 1
        return cond, ipiv

    def _lu_step(self, st: _Step, mine, ipiv):
        A, ctx, k = self.A, self.ctx, st.k
        if ctx.rank == st.owner:
            buf, view, _, _, _, _ = mine
            r0 = 0
            for m, r in zip(st.dom, st.rows):
                A.tile(m, k).copy_(view[r0:r0 + r])
                r0 += r
        if self.IPIV.is_local(k, k):
            t = self.IPIV.tile(k, k)
            t.zero_()
            t[:st.kmax, 0] = torch.from_numpy(ipiv + 1).to(torch.int32).to(t.device)
        # row interchanges inside the domain stack of the trailing columns (all on k's process row)
        perm = _perm_from_swaps(ipiv, st.M)
        mv = np.nonzero(perm != np.arange(st.M))[0]
        trail = [n for n in range(k + 1, A.nt) if A.col_is_local(n)]
        _permute_rows_2d(ctx, A, st.grow[mv], st.grow[perm[mv]], trail)
        if ctx.world == 1:
            self._lu_update_local(st)
            return
        self._lu_update_prog(st)

    def _lu_update_local(self, st: _Step):
        """One process: the LU step's solves and trailing update as three batched launches (TRSM of
        row k with L_kk, TRSM of the off-domain tiles with U_kk, one MFMA GEMM batch built with numpy),
        cached per step across runs -- no per-tile program construction on the critical path."""
        A, k = self.A, st.k
        b = self._lu_batches.get(k)
        if b is None:
            kb = A.tile_cols(k)
            dkk = A.offset(k, k)
            row = TileBatch()
            for n in range(k + 1, A.nt):
                row.add(dkk, A.tile_rows(k), A.tile_cols(n), b_off=A.offset(k, n))
            off = TileBatch()
            for m in st.off:
                off.add(dkk, A.tile_rows(m), kb, b_off=A.offset(m, k))
            gb = None
            if k + 1 < A.mt and k + 1 < A.nt:
                ms = np.arange(k + 1, A.mt)
                ns = np.arange(k + 1, A.nt)
                ro = np.array([A.offset(m, k) for m in ms], dtype=np.int64)      # column k of every row
                co = np.array([A.offset(k, n) for n in ns], dtype=np.int64)      # row k of every column
                cbase = np.array([A.offset(m, k + 1) for m in ms], dtype=np.int64)
                dcol = co - co[0]                                                 # tile-column stride
                mm, nn = np.meshgrid(np.arange(len(ms)), np.arange(len(ns)), indexing="ij")
                c_off = cbase[mm] + dcol[nn]
                rows = np.array([A.tile_rows(m) for m in ms], dtype=np.int64)[mm]
                cols = np.array([A.tile_cols(n) for n in ns], dtype=np.int64)[nn]
                gb = GemmBatch().add_arrays(c_off, rows, cols, 1, ro[mm], co[nn], kb).finalize()
            b = self._lu_batches[k] = (row.finalize() if len(row) else None, off.finalize() if len(off) else None,
                                       gb)
        row, off, gb = b
        if row is not None:
            ops.trsm(dplasmaLeft, dplasmaLower, N_, dplasmaUnit, 1.0, A.data, A.ld, A.data, A.ld, row)
        if off is not None:
            ops.trsm(dplasmaRight, dplasmaUpper, N_, dplasmaNonUnit, 1.0, A.data, A.ld, A.data, A.ld, off)
        if gb is not None:
            ops.gemm(N_, N_, -1.0, A.data, A.ld, A.data, A.ld, 1.0, A.data, A.ld, gb)

    def _qr_step(self, st: _Step, zero_ipiv: bool = True):
        A, ctx, k = self.A, self.ctx, st.k
        if zero_ipiv and self.IPIV.is_local(k, k):
            self.IPIV.tile(k, k).zero_()
        f = self.qpf
        if f is not None:
            if f.simple:
                e = f.steps[k][0]
                f.panel(k, e, 0)
                f.apply(e, e.get("next"), 0, f.wn)
                f.apply(e, e.get("rest"), 0, f.wr)
            elif f.batched:
                f.step_batched(k)
            else:
                f.step_general(k)
            return
        dag = TileDAG(ctx, f"getrf_qrf_qr({k})")
        qr._factor(dag, qr._L(A), qr._L(self.TS), qr._L(self.TT), self.kd, self.tree, ks=[k])
        dag.compile().execute(ctx)

    def run(self, ctx=None):
        import time
        self._t_run = time.perf_counter()
        A = self.A
        ctx = self.ctx
        if self.fast is not None:
            if self.tasks:
                Taskpool.run(self, ctx)
            else:
                self._run_fast()
            if self.info_out is not None:
                self.info_out[0] = 0
            return
        if self.devcrit:
            self._run_devcrit()
            if self.info_out is not None:
                self.info_out[0] = 0
            return
        if self.devcrit_dist:
            self._run_devcrit_dist()
            if self.info_out is not None:
                self.info_out[0] = 0
            return
        for k in range(self.minMNT):
            st = _Step(A, k, self.p)
            mine = self._domain_lu(st) if ctx.rank == st.owner else None
            cond, ipiv = self._decide(st, mine)
            self.lu_tab[k] = cond
            if cond:
                self._lu_step(st, mine, ipiv)
            else:
                self._qr_step(st)
        if self.info_out is not None:
            self.info_out[0] = 0

    def complete(self, ctx=None):
        if self.ctx.is_gpu:
            torch.cuda.current_stream(self.ctx.device).synchronize()
        if self.qpf is not None and int(self.qpf.info.item()) != 0:
            raise RuntimeError(f"getrf_qrf: QR panel kernel reported {int(self.qpf.info.item())}")
        r = int(self.fast_info.item()) if self.fast is not None else 0
        if (self.devcrit or self.devcrit_dist) and self._dec:
            # the decisions, read back once for the whole factorisation
            dec = torch.cat(self._dec).cpu().tolist()
            for k, c in enumerate(dec):
                self.lu_tab[k] = int(c)
            if "_dinfo" in self.__dict__ and int(self._dinfo.item()) != 0:
                raise RuntimeError(f"getrf_qrf: row interchanges reported {int(self._dinfo.item())}")
        if self.info_out is not None:
            self.info_out[0] = r
        self._result = r
        return r


def getrf_qrf_New(ctx, qrtree_, A, IPIV, TS, TT, criteria=DEFAULT_CRITERIUM, alpha=1.0, lu_tab=None, INFO=None,
                  p=None):
    """Hybrid LU-QR factorization (dplasma_zgetrf_qrf_New).  ``p``: domain period (default: grid rows)."""
    qr._check_square_tiles(A)
    if TS.nb != A.nb or TT.nb != A.nb:
        raise ValueError("TS/TT must have tiles of ib x nb")
    return _GetrfQrf(ctx, qrtree_, A, IPIV, TS, TT, criteria, alpha, lu_tab, INFO, p)


def getrf_qrf(ctx, qrtree_, A, IPIV, TS, TT, criteria=DEFAULT_CRITERIUM, alpha=1.0, lu_tab=None, INFO=None, p=None):
    getrf_qrf_New(ctx, qrtree_, A, IPIV, TS, TT, criteria, alpha, lu_tab, INFO, p).execute(ctx)
    return 0


def trsmpl_qrf(ctx, qrtree_, A, IPIV, B, TS, TT, lu_tab, p=None):
    """Apply the hybrid factorization's L / Q^H to B: B := (L_k or Q_k)^-1 ... B (dplasma_ztrsmpl_qrf);
    then solve with the upper triangle of A (trsm Left Upper NoTrans NonUnit) to get x."""
    p = p or A.grid.P
    kd = qr_ops.kinds(A.dtype, TS.mb, (0, 0), (0, 0))
    ap = None
    if getattr(TS, "qr_format", "tile") == "panel":
        # QR steps factored by the stacked-domain engine: apply Q_k^H in its format, item by item
        ap = qr_panel._Apply(ctx, dplasmaLeft, dplasmaConjTrans, A, TS, TT, B, qrtree_)
        byk = {}
        for it in ap.items:
            byk.setdefault(it["k"], []).append(it)
    for k in range(min(A.mt, A.nt)):
        if not lu_tab[k] and ap is not None:
            for it in byk.get(k, ()):
                ap.run_item(it)
        elif lu_tab[k]:
            st = _Step(A, k, p)
            piv = torch.zeros(A.mb, dtype=torch.float64)
            if IPIV.is_local(k, k):
                piv[:] = IPIV.tile(k, k)[:, 0].double().cpu()
            if ctx.world > 1:
                d = piv.to(ctx.device)
                comm.allreduce(d)
                piv = d.cpu()
            ipiv = piv[:st.kmax].round().to(torch.int64).numpy() - 1
            perm = _perm_from_swaps(ipiv, st.M)
            mv = np.nonzero(perm != np.arange(st.M))[0]
            cols = [n for n in range(B.nt) if B.col_is_local(n)]
            _permute_rows_2d(ctx, B, st.grow[mv], st.grow[perm[mv]], cols)
            prog = TileProgram(ctx, f"trsmpl_qrf_lu({k})")
            s = prog.stage("trsm")
            for n in range(B.nt):
                s.trsm(dplasmaLeft, dplasmaLower, N_, dplasmaUnit, 1.0, (A, k, k), (B, k, n))
            if k + 1 < B.mt:
                s = prog.stage("gemm")
                for m in range(k + 1, B.mt):
                    for n in range(B.nt):
                        s.gemm((B, m, n), [((A, m, k), N_, (B, k, n), N_)], alpha=-1.0, beta=1.0)
            prog.compile().execute(ctx)
        else:
            dag = TileDAG(ctx, f"trsmpl_qrf_qr({k})")
            qr._apply(dag, qr._L(A), qr._L(TS), qr._L(TT), qr._L(B), kd, True, qrtree_, ks=[k])
            dag.compile().execute(ctx)
    return 0


def trsmpl_qrf_New(ctx, qrtree_, A, IPIV, B, TS, TT, lu_tab, p=None) -> Taskpool:
    tp = Taskpool("trsmpl_qrf", ctx)
    tp.task("trsmpl_qrf", "update", lambda: trsmpl_qrf(ctx, qrtree_, A, IPIV, B, TS, TT, lu_tab, p))
    return tp.finish_build()


def gesv_qrf(ctx, qrtree_, A, IPIV, TS, TT, B, criteria=DEFAULT_CRITERIUM, alpha=1.0, p=None):
    """Convenience driver: hybrid factorization + solve (as tests/testing_zgetrf_qrf.c checks it)."""
    from . import blas3
    lu_tab = [0] * min(A.mt, A.nt)
    getrf_qrf(ctx, qrtree_, A, IPIV, TS, TT, criteria, alpha, lu_tab, None, p)
    trsmpl_qrf(ctx, qrtree_, A, IPIV, B, TS, TT, lu_tab, p)
    blas3.trsm(ctx, dplasmaLeft, dplasmaUpper, N_, dplasmaNonUnit, 1.0, A, B)
    return lu_tab
