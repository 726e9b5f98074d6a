"""LU factorizations and solves.

Reference: ``src/zgetrf_nopiv.jdf`` (zgetrf_nopiv(k) :46, ztrsm_l :86, ztrsm_u
:128, zgemm :169), ``src/zgetrf_1d.jdf`` (partial pivoting with a
multithreaded panel, :70-359; ``src/zgetrf_1d_wrapper.c:82``), ``src/zlaswp.jdf``
/ ``zlaswp_wrapper.c`` and the ScaLAPACK-style drivers getrs / gesv.

MI355X design:
* getrf_nopiv: TileProgram stages per step (tile LU kernel, two batched TRSM
  launches, one MFMA GEMM launch) on any P x Q grid.
* getrf_1d (partial pivoting): 1-D block-cyclic column distribution (P = 1,
  exactly the reference's "1d" variant): the panel's owner assembles the tile
  column into one contiguous tall panel, factors it with the pivoting panel
  kernel (workgroup-wide argmax in LDS), and broadcasts factor + pivots to the
  other ranks; every rank applies the net row permutation to its local columns
  with two row-gather launches, then one TRSM launch and one MFMA GEMM launch
  update its trailing tiles.  Pivots are returned LAPACK-style (global,
  1-based, sequential interchanges) in a 1 x min(M,N) IPIV descriptor.
"""
from __future__ import annotations

import bisect
import os

import numpy as np
import torch

from ..constants import (DPLASMA_ERR_NOT_SUPPORTED, dplasmaLeft, dplasmaLower, dplasmaNoTrans, dplasmaNonUnit,
                         dplasmaRight, dplasmaTrans, dplasmaConjTrans, dplasmaUnit, dplasmaUpper)
from ..descriptor import TiledMatrix
from ..ops import tile_ops as ops
from ..ops import lu_dist_ops
from ..ops.batch import GemmBatch, TileBatch
import torch.distributed as dist

from ..parallel import comm
from ..runtime import Taskpool
from ..runtime.tileprog import TileProgram
from ..utils.flops import flops
from . import blas3

N_ = dplasmaNoTrans


# ----------------------------------------------------------------------------- no pivoting
def _tile_lu_nopiv(A, key, info, base):
    def fn(res):
        b, off, ld = res[key]
        m, n = A.tile_rows(key[1]), A.tile_cols(key[2])
        ops.getrf_panel(b, off, m, n, ld, None, info, base, pivot=False)
    return fn


def getrf_nopiv_New(ctx, A, info_out=None):
    """LU without pivoting (dplasma_zgetrf_nopiv_New, src/zgetrf_nopiv.jdf): the partial-pivoting
    engine's PANEL / SWAP / NEXT / REST task structure with a non-pivoting panel (recursive device
    LU on the tall panel, one TRSM launch for the U block row, MFMA GEMM trailing updates) on square
    tiles; other tilings run the tile program below."""
    if A.mb != A.nb:
        return _getrf_nopiv_tiles_New(ctx, A, info_out)
    tp = Taskpool("getrf_nopiv", ctx)
    tp.flops = flops(A.prec, "getrf", A.m, A.n)
    info = torch.zeros(1, dtype=torch.int32, device=A.device)
    st = _GetrfDev(ctx, A, info, pivot=False)
    st.add_tasks(tp, "getrf_nopiv")
    tp._state = st
    tp.info = info

    def _done():
        r = _reduce_info(info)
        if info_out is not None:
            info_out[0] = r
        return r
    tp.on_complete(_done)
    return tp.finish_build()


def _getrf_nopiv_tiles_New(ctx, A, info_out=None):
    prog = TileProgram(ctx, "getrf_nopiv")
    prog.flops = flops(A.prec, "getrf", A.m, A.n)
    info = torch.zeros(1, dtype=torch.int32, device=A.device)
    kt = min(A.mt, A.nt)
    for k in range(kt):
        s = prog.stage(f"getrf({k})")
        s.batch_fn([(A, k, k)], [], _tile_lu_nopiv(A, (prog.mid(A), k, k), info, k * A.mb))
        s = prog.stage(f"trsm({k})")
        for m in range(k + 1, A.mt):
            s.trsm(dplasmaRight, dplasmaUpper, N_, dplasmaNonUnit, 1.0, (A, k, k), (A, m, k))
        for n in range(k + 1, A.nt):
            s.trsm(dplasmaLeft, dplasmaLower, N_, dplasmaUnit, 1.0, (A, k, k), (A, k, n))
        s = prog.stage(f"gemm({k})")
        for m in range(k + 1, A.mt):
            for n in range(k + 1, A.nt):
                s.gemm((A, m, n), [((A, m, k), N_, (A, k, n), N_)], alpha=-1.0, beta=1.0)
    tp = prog.compile()
    tp.info = info

    def _done():
        v = info.clone()
        comm.allreduce(v, op=torch.distributed.ReduceOp.MAX)
        r = int(v.item())
        if info_out is not None:
            info_out[0] = r
        return r
    tp.on_complete(_done)
    return tp


def getrf_nopiv(ctx, A):
    return getrf_nopiv_New(ctx, A).execute(ctx)


# ----------------------------------------------------------------------------- pivot helpers
def ipiv_descriptor(ctx, A, name="IPIV") -> TiledMatrix:
    """1 x min(M,N) int32 descriptor (tiles 1 x nb) on the context grid."""
    k = min(A.m, A.n)
    return TiledMatrix(torch.int32, 1, A.nb, 1, k, P=1, Q=ctx.world, rank=ctx.rank, device=A.device, name=name)


def _perm_from_swaps(piv: np.ndarray, nrows: int) -> np.ndarray:
    """Sequential interchanges i <-> piv[i] (0-based, rows of a panel) -> perm with new[r] = old[perm[r]]."""
    perm = np.arange(nrows)
    for i, p in enumerate(piv):
        if p != i:
            perm[i], perm[p] = perm[p], perm[i]
    return perm


def _row_pairs(M: TiledMatrix, rows_dst, rows_src, coltiles, dst_off_fn=None, src_off_fn=None):
    """RowPair records for rows (global element row indices) across the given local column tiles."""
    out = []
    for n in coltiles:
        for d, s in zip(rows_dst, rows_src):
            od = dst_off_fn(d, n) if dst_off_fn else M.offset(d // M.mb, n) + d % M.mb
            os_ = src_off_fn(s, n) if src_off_fn else M.offset(s // M.mb, n) + s % M.mb
            out.append((od, os_))
    return np.array(out, dtype=ops.ROW_PAIR)


class _GetrfDev:
    """Partial-pivoting LU, device-resident (getrf_1d on 1 x Q grids, getrf_ptgpanel on P x Q).

    Step k is four tasks (every batch and panel plan is built once, here; a run only launches):
      PANEL(k)  [panel stream]  the panel's process column gathers the tall panel -- each process
                row contributes only its own tiles (one all-gather of M x NB / P per rank instead
                of the former all-reduce of the whole zero-padded panel) -- and factors it with the
                recursive device LU (ops.PanelLU: dgetrf2 halves, <=64-column blocks with an
                on-device multi-workgroup pivot search -- GETRF_MAX / RDC / SND of
                src/zgetrf_ptgpanel.jdf:206-590), then factored panel + pivots travel along
                process rows (RCCL broadcast);
      SWAP(k)   [update stream] net row moves derived on the device (ops.piv_moves) applied to every
                local tile column (SWAP_COLLECT / SWAP_SND, :825-978; summed over the process column
                when P > 1), L written back, the U block row solved where it lives and broadcast
                down process columns;
      NEXT(k)   [panel stream]  the trailing update of tile column k+1 only;
      REST(k)   [update stream] the trailing update of every column beyond it.
    PANEL(k+1) needs only NEXT(k), so with look-ahead (DPLASMA_LU_LOOKAHEAD=1) the next panel
    factorisation overlaps REST(k) -- the reference's lookahead through priorities.  Panel buffers alternate with k's parity (REST(k) still reads panel k).

    Panel modes for P > 1 (``DPLASMA_LU_PANEL``):
      "dist" -- the reference's distributed pivoting on the GPUs (ops.lu_dist_ops): each
               process row keeps its own panel rows plus a replica of the diagonal tile rows, and
               every column's pivot is chosen inside the persistent panel kernel through one
               cross-process hand-off (IPC-mapped exchange buffers over xGMI, epoch flags): O(NB^2)
               elements per rank and panel instead of the whole panel, no host round trip;
      "gather" (default) -- the panel's process column exchanges its tiles point to point (exact per-step
               sizes) and every process row factors the tall panel redundantly with the one-process tagged
               panel kernel (O(M NB / P) elements per rank, no per-column cross-process hand-off);
      "percol" -- the distributed pivoting driven from the host (one all-gather and two host
               syncs per column; kept as the transport-independent reference of "dist")."""

    def __init__(self, ctx, A, info, pivot: bool = True, trailing_only: bool = False, lookahead=None,
                 panel_bw=None):
        self.ctx, self.A, self.info = ctx, A, info
        self.pivot = pivot   # False: getrf_nopiv (same task structure, no interchanges)
        # trailing_only: step k's interchanges touch tile columns >= k only (the hybrid LU-QR keeps every
        # earlier step's factor in its own row order, models/lu_qr.py)
        self.trailing_only = trailing_only
        dev = self.dev = A.device
        mb, nb = A.mb, A.nb
        g = A.grid
        self.kt = min(A.mt, A.nt)
        # round 2: look-ahead opt-in -- measured on one MI355X (profiles/r2_lu_lookahead.txt) the persistent
        # grid-barrier panel kernel beside the REST GEMM slows from ~0.5 to ~1.2 ms per 64-column
        # block (its workgroups share CUs with GEMM waves), which eats the overlap: DGETRF 32k
        # 28.2 -> 27.1 TF/s, 64k 48.1 -> 47.2 TF/s with look-ahead on
        # (lookahead=True: a caller that issues PANEL(k+1) beside REST(k) itself -- the hybrid LU-QR -- needs the
        # parity-alternating panel buffers whatever the environment says)
        # P > 1 with the point-to-point interchanges: look-ahead on by default -- the distributed panel's per-column
        # cross-process hand-offs are latency, not CU time, so they belong beside the bulk update (tools/replay_lu.py)
        la_def = "1" if (g.P > 1 and pivot and os.environ.get("DPLASMA_LU_PANEL", "gather") != "percol"
                         and os.environ.get("DPLASMA_LU_XROWS", "p2p") != "allreduce") else "0"
        # one process, round 6: re-measured with the tagged pivoting kernel and the deferred left interchanges, look-ahead
        # with 32-column pivoting blocks (64 KB of LDS: room for a GEMM workgroup beside it) now wins -- 32k 35.1-35.2
        # -> 36.0, 64k 53.7 -> 54.0 TF/s (tools/gpu/r6_b29.sh; r6_b19 without the deferral: 34.2 -> 35.3, 53.2 -> 53.6)
        la_p1 = g.P == 1 and g.Q == 1 and pivot and lookahead is None and "DPLASMA_LU_LOOKAHEAD" not in os.environ
        if la_p1:
            la_def = "1"
            if panel_bw is None and "DPLASMA_LU_BW" not in os.environ:
                panel_bw = 32
        self.lookahead = (os.environ.get("DPLASMA_LU_LOOKAHEAD", la_def) == "1") if lookahead is None else bool(lookahead)
        self.panel_bw = panel_bw   # base block width of the recursive panel (None: ops.LU_BW)
        self.pbufs = [torch.zeros(max(1, A.m * nb), dtype=A.dtype, device=dev)
                      for _ in range(2 if self.lookahead else 1)]
        self.piv_dev = torch.zeros(nb, dtype=torch.int32, device=dev)
        self.ipiv_all = torch.zeros(max(1, min(A.m, A.n)), dtype=torch.int32, device=dev)
        self.ws = ops.lu_workspace(A.m, dev)
        # gather (default): measured in the 2 x 4 rank replay against the distributed-pivoting kernel (its per-column
        # grid barrier + cross-rank hand-off is 12-17 us per column against the one-process tagged panel's ~5,
        # tools/gpu/lu_xlat_probe.py, profiles/r6_lu_config5.txt); the pivots are the same
        self.panel_mode = os.environ.get("DPLASMA_LU_PANEL", "gather")
        if self.panel_mode not in ("dist", "gather", "percol"):
            raise ValueError(f"DPLASMA_LU_PANEL={self.panel_mode!r}: expected dist, gather or percol")
        self.percol = self.panel_mode == "percol" and g.P > 1 and pivot
        self.dist = self.panel_mode == "dist" and g.P > 1 and pivot and A.mb == A.nb
        self.xc = None
        if self.dist:
            # exchange buffers of my process column (every rank of the column creates them together)
            # largest (diagonal replica + own rows) panel any rank factors -- the same number on every rank
            per_row = [0] * g.P
            for m in range(A.mt):
                per_row[g.prow(m + A.it0)] += A.tile_rows(m)
            self.xc = lu_dist_ops.panel_xchg(ctx.col_group, A.myrow, g.P, nb, A.dtype, dev, max(per_row) + mb)
            self.dws = lu_dist_ops.dist_workspace(nb, dev)
            self.tbuf = torch.zeros(max(1, mb * nb), dtype=A.dtype, device=dev)
        self.cnt = torch.zeros(1, dtype=torch.int32, device=dev)
        # move lists double-buffered by step parity: step k+2 must not overwrite the lists the
        # side stream is still applying to the left (already factored) columns of step k
        self.mdst = torch.zeros(2, 2 * nb, dtype=torch.int32, device=dev)
        self.msrc = torch.zeros(2, 2 * nb, dtype=torch.int32, device=dev)
        self.mcnt = torch.zeros(2, 1, dtype=torch.int32, device=dev)
        # row / column offset tables of the local tiles (offset(m, n) = rowoff[m] + coloff[n])
        lrows = [m for m in range(A.mt) if A.row_is_local(m)]
        lcols = [n for n in range(A.nt) if A.col_is_local(n)]
        self.lcols = lcols
        if lrows and lcols:
            mr, nr = lrows[0], lcols[0]
            base = A.offset(mr, nr)
            rowoff = [A.offset(m, nr) - base if A.row_is_local(m) else -1 for m in range(A.mt)]
            coloff = [A.offset(mr, n) for n in lcols]
            self.rowoff = torch.tensor(rowoff, dtype=torch.int64, device=dev)
            self.coloff = torch.tensor(coloff, dtype=torch.int64, device=dev)
            self.ncols = torch.tensor([A.tile_cols(n) for n in lcols], dtype=torch.int32, device=dev)
            width = len(lcols) * nb
            self.tmp = torch.zeros(2 * nb * width, dtype=A.dtype, device=dev)
        else:
            self.rowoff = self.coloff = self.ncols = self.tmp = None
        # P == 1, opt-in (DPLASMA_LU_SIDE_SWAPS=1): the interchanges of the already factored
        # columns (tile columns < k) are off the critical path -- only LAPACK's final L needs
        # them -- so they can run on a low-priority side stream (zgetrf_1d.jdf applies them as
        # separate SWAP tasks).  Measured on one MI355X (profiles/r1_lu_side_swaps.txt): the
        # split moves contend with the trailing GEMM and the persistent panel kernel, the sum of
        # row-move time grows 82 -> 132 ms at N=32k and the factorisation is no faster, so the
        # default keeps one exchange per step.  P > 1 always keeps one summed exchange.
        self.inplace_moves = os.environ.get("DPLASMA_LU_INPLACE_MOVES", "1") != "0"
        # P == 1 (DPLASMA_LU_DEFER_LEFT, default on: 32k 34.4 -> 35.1, 64k 52.7 -> 53.6 TF/s, r6_b28): every step's interchanges touch the trailing columns only, and each factored
        # tile column gets the composition of all later steps' interchanges once, at the end (piv_compose_left +
        # rows_perm_col): each left element moves once instead of once per later step, off the steps' critical path
        # (the reference's swpback(k, n) tasks, priority 0, chained per left column: src/zgetrf_1d.jdf:360-409)
        # (not with DPLASMA_LU_SIDE_SWAPS=1, which applies the same left moves step by step on a side stream)
        self.defer_left = (self.tmp is not None and A.grid.P == 1 and pivot and not trailing_only
                           and os.environ.get("DPLASMA_LU_SIDE_SWAPS", "0") != "1"
                           and os.environ.get("DPLASMA_LU_DEFER_LEFT", "1") == "1")
        if self.defer_left:
            self.trailing_only = True
            self.coloff_h = [A.offset(lrows[0], n) for n in lcols]
        self.side = None
        if self.tmp is not None and A.grid.P == 1 and dev.type == "cuda" and \
                os.environ.get("DPLASMA_LU_SIDE_SWAPS", "0") == "1":
            self.side = torch.cuda.Stream(device=dev, priority=0)
            self.tmp_l = torch.zeros_like(self.tmp)
            self.ev_side = [None, None]
        self.nleft = [bisect.bisect_left(lcols, k) for k in range(min(A.mt, A.nt))]
        # P > 1 (DPLASMA_LU_XROWS=p2p, the default): the interchanges move only the rows whose source and destination
        # lie on different process rows, point to point inside the process column (the reference's SWAP_COLLECT /
        # SWAP_SND, src/zgetrf_ptgpanel.jdf:825-984), classified on the device from the move list (no host pivots),
        # and split by urgency: the next panel's column (panel stream, urgent communicator), the rest of the trailing
        # columns (update stream) and the already factored columns (low-priority side stream -- only the final L
        # needs them).  "allreduce" keeps round 5's summed exchange of the whole 2 NB-row staging buffer.
        self.xmode = (g.P > 1 and pivot and not self.percol and bool(lcols) and
                      os.environ.get("DPLASMA_LU_XROWS", "p2p") != "allreduce")
        self.nch = 1
        # gather-mode panels on P x Q grids: the panel's tiles travel point to point with the exact per-step sizes
        # (packed slots; an all-gather would move the largest step's slot every step), and with DPLASMA_LU_RNF=1
        # the ranks of the NEXT panel's process column receive them too and factor panel k redundantly -- the
        # factored panel then never travels on the critical path, NEXT(k) runs on a column that factored it (off by
        # default: the rank replay charges the extra factorisation and cannot credit the cross-rank chain it
        # shortens, profiles/r6_lu_config5.txt)
        self.gxp2p = g.P > 1 and pivot and self.panel_mode == "gather"
        # RNF is switched off: the 2 x 4 one-GPU rehearsal gives wrong factors (correct pivots) with it, before and after
        # the round-6 LSEND buffer fix (tools/gpu/r6_b27.sh) -- DPLASMA_LU_RNF=1 is ignored with a warning until fixed
        # (r6 debug run: the wrong tiles are the left (already factored) columns of the redundant-factorising process
        # column, rows moved by late steps -- its LEFT interchanges).  The cross-stream hazard checker
        # (tests/test_lu_hazards.py) finds no scratch-buffer race with RNF forced on; tracking the matrix storage by
        # element span flags the same pairs with and without RNF (tile spans overlap), so the cause is still open
        self.rnf = False
        if self.gxp2p and self.xmode and g.Q > 1 and os.environ.get("DPLASMA_LU_RNF", "0") == "1":
            import warnings
            warnings.warn("DPLASMA_LU_RNF=1 ignored: the redundant next-column panel factorisation is disabled "
                          "(wrong factors in the 2x4 rehearsal)")
        if self.xmode:
            # the rest of the trailing columns in DPLASMA_LU_CHUNKS column chunks: chunk c's interchanges / U block of
            # step k+1 (exchange stream) overlap the update of chunk c+1 of step k (update stream)
            self.nch = max(1, int(os.environ.get("DPLASMA_LU_CHUNKS", "2")))
            if dev.type == "cuda" and "xch" not in ctx.streams:
                ctx.streams["xch"] = torch.cuda.Stream(device=dev, priority=torch.cuda.Stream.priority_range()[1])
            self.xpeers = [q for q in range(g.P) if q != A.myrow]
            self.prow_t = torch.tensor([g.prow(m + A.it0) for m in range(A.mt)], dtype=torch.int32, device=dev)
            self.xo = torch.full((2, 2 * nb), -1, dtype=torch.int32, device=dev)
            wtot = len(lcols) * nb

            def xbufs(W):
                sb = {q: torch.zeros(max(1, nb * W), dtype=A.dtype, device=dev) for q in self.xpeers}
                rb = {q: torch.zeros(max(1, nb * W), dtype=A.dtype, device=dev) for q in self.xpeers}
                if dev.type == "cuda":
                    sp = torch.tensor([sb[q].data_ptr() if q in sb else 0 for q in range(g.P)], dtype=torch.int64,
                                      device=dev)
                    rp = torch.tensor([rb[q].data_ptr() if q in rb else 0 for q in range(g.P)], dtype=torch.int64,
                                      device=dev)
                else:
                    sp, rp = [sb.get(q) for q in range(g.P)], [rb.get(q) for q in range(g.P)]
                return {"send": sb, "recv": rb, "sp": sp, "rp": rp}
            self.xb = {"next": xbufs(nb), "rest": xbufs(wtot)}
            # SWAPN (panel stream) stages the next column's moved rows in a buffer of its own: sharing self.tmp with
            # the SWAPR chunks (exchange stream) let a chunk's gather overwrite rows SWAPN had not scattered yet --
            # the two tasks of a step have no edge between them
            self.tmp_n = torch.zeros(2 * nb * nb, dtype=A.dtype, device=dev) if self.tmp is not None else None
            if not trailing_only:
                self.xb["left"] = xbufs(wtot)
                self.tmp_x = torch.zeros_like(self.tmp) if self.tmp is not None else None
            self.g_next = ctx.urgent_group if ctx.urgent_group is not None else ctx.col_group
            bulk = list(ctx.bulk_groups) or [ctx.col_group]
            self.g_rest, self.g_left = bulk[0], bulk[-1]
        elif self.gxp2p:
            # gather panels with the summed row exchange (DPLASMA_LU_XROWS=allreduce): the panel slots still travel
            # point to point, on the urgent communicator
            self.g_next = ctx.urgent_group if ctx.urgent_group is not None else ctx.col_group
        ncol_loc = sum(A.tile_cols(n) for n in lcols)
        self.ubuf = torch.zeros(max(1, nb * max(ncol_loc, 1)), dtype=A.dtype, device=dev)
        # xmode: U blocks double-buffered by step parity (step k+1's exchanges run while step k's update chunks read)
        self.ubufs = [self.ubuf, torch.zeros_like(self.ubuf) if self.xmode else self.ubuf]
        # P > 1: per-step panel gather buffer [P][maxrows x nb] (every process row's panel tiles)
        self.gbuf = None
        if g.P > 1 and not self.dist and not self.percol:
            maxrows = 0
            for k in range(self.kt):
                for q in range(g.P):
                    maxrows = max(maxrows, sum(A.tile_rows(m) for m in range(k, A.mt) if g.prow(m + A.it0) == q))
            self.gmax = max(1, maxrows)
            self.gbuf = torch.zeros(g.P * self.gmax * nb, dtype=A.dtype, device=dev)
        # P > 1 panel mode: "gather" (default) -- the panel's process column all-gathers the tall panel
        # and every process row factors it redundantly (one collective per panel); "percol" -- the
        # reference's distributed pivoting (zgetrf_ptgpanel.jdf GETRF_MAX / RDC / SND): each process
        # row keeps its own panel rows, every column's pivot is chosen by one small all-gather of the
        # local candidates (value, row, candidate row, current diagonal row) and only the two rows of
        # an interchange move; O(NB (NB + P)) elements per panel instead of O(M NB / P)
        self.plan = [self._build(k) for k in range(self.kt)]
        rl = max([st.get("rlen", 0) for st in self.plan] + [0])
        self.rbuf = torch.zeros(max(1, rl), dtype=A.dtype, device=dev) if rl else None
        # LSEND: the panel's row transfers as a task of their own (look-ahead, gather panels on P x Q); the pivots
        # travel from a copy (piv_dev is re-filled by the next panel while the send may still be in flight)
        self.lsend_task = bool(self.lookahead and self.xmode and self.gxp2p and g.Q > 1)
        self.piv_send = [torch.zeros_like(self.piv_dev), torch.zeros_like(self.piv_dev)]
        # ... and the rows from their own buffers (by step parity): rbuf is this rank's RECEIVE buffer of the next steps
        # (PANEL(k+1) on a rank of panel k's column receives there while LSEND(k) may still be packing / sending --
        # no task edge orders the two; sharing rbuf gave intermittently wrong factors with correct pivots)
        self.rbuf_send = ([torch.zeros_like(self.rbuf), torch.zeros_like(self.rbuf)]
                          if (self.lsend_task and self.rbuf is not None) else None)
        if self.lsend_task and dev.type == "cuda" and "lsend" not in ctx.streams:
            ctx.streams["lsend"] = torch.cuda.Stream(device=dev, priority=torch.cuda.Stream.priority_range()[1])
        self.bytes_panel = [0] * self.kt   # elements this rank sends per step (panel exchange)
        if self.percol:
            mlmax = max([st.get("Ml", 0) for st in self.plan] + [1])
            self.lpbuf = torch.zeros(mlmax * nb, dtype=A.dtype, device=dev)
            self.xbuf = torch.zeros(g.P * (2 + 2 * nb), dtype=A.dtype, device=dev)

    def _build(self, k):
        A = self.A
        mb = A.mb
        kb = A.tile_cols(k)
        r0 = k * mb
        mp = A.m - r0
        st = {"kb": kb, "r0": r0, "mp": mp, "kmin": min(mp, kb)}
        g = A.grid
        st["pv"] = self.pbufs[k % len(self.pbufs)]
        # panel buffer layout: row offset of tile row m's L(m, k) and the buffer's leading dimension
        if self.dist:
            # [T: replica of the diagonal tile rows][my own tiles below it]
            tr = A.tile_rows(k)
            own = [m for m in range(k + 1, A.mt) if A.row_is_local(m)]
            lay, r, lrel = {k: 0}, tr, []
            for m in own:
                lay[m] = r
                lrel.extend(range((m - k) * mb, (m - k) * mb + A.tile_rows(m)))
                r += A.tile_rows(m)
            st["pld"], st["tr"] = r, tr
        else:
            lay = {m: (m - k) * mb for m in range(k, A.mt)}
            st["pld"] = mp
            if g.P > 1 and g.Q > 1 and self.gbuf is not None:
                # the row broadcast of the factored panel carries this process row's tiles only (the row peers'
                # trailing updates read nothing else): packed by the root, unpacked at the same place by the others
                mine_r = [m for m in range(k, A.mt) if A.row_is_local(m)]
                pk, upk, r = TileBatch(), TileBatch(), 0
                for m in mine_r:
                    pk.add(lay[m], A.tile_rows(m), kb, b_off=r)
                    upk.add(r, A.tile_rows(m), kb, b_off=lay[m])
                    r += A.tile_rows(m)
                st["rlen"], st["rld"] = r * kb, max(1, r)
                if r:
                    st["rpack"], st["runpack"] = pk.finalize(), upk.finalize()
        if A.col_is_local(k) and self.dist:
            diag = A.row_is_local(k)
            tb, back = TileBatch(), TileBatch()
            for m in ([k] if diag else []) + own:
                tb.add(A.offset(m, k), A.tile_rows(m), kb, b_off=lay[m])
                back.add(lay[m], A.tile_rows(m), kb, b_off=A.offset(m, k))
            st["gather"], st["back"] = tb.finalize(), back.finalize()
            if diag:
                st["tpack"] = TileBatch().add(A.offset(k, k), tr, kb, b_off=0).finalize()
            else:
                st["tunpack"] = TileBatch().add(0, tr, kb, b_off=0).finalize()
            st["plu"] = lu_dist_ops.DistPanelLU(st["pv"], r, r, kb, tr, diag, lrel)
            st["kmin"] = min(st["kmin"], tr)
            self.bytes_panel_plan = getattr(self, "bytes_panel_plan", {})
            self.bytes_panel_plan[k] = st["kmin"] * (2 + kb) * (g.P - 1)
        elif A.col_is_local(k) or (self.rnf and k + 1 < A.nt and A.col_is_local(k + 1)):
            own_col = A.col_is_local(k)
            st["fac"] = True
            mine = [m for m in range(k, A.mt) if A.row_is_local(m)]
            if mine and own_col:
                tb, back = TileBatch(), TileBatch()
                for m in mine:
                    tb.add(A.offset(m, k), A.tile_rows(m), kb, b_off=(m - k) * mb)
                    back.add((m - k) * mb, A.tile_rows(m), kb, b_off=A.offset(m, k))
                st["gather"], st["back"] = tb.finalize(), back.finalize()
            if self.gxp2p:
                # exact slots: process row q's tiles of the panel, packed (ld = its row count) one after another
                rows_q = [sum(A.tile_rows(m) for m in range(k, A.mt) if g.prow(m + A.it0) == q) for q in range(g.P)]
                off_q = [sum(rows_q[:q]) * kb for q in range(g.P)]
                pack, unpack = TileBatch(), [TileBatch() for _ in range(g.P)]
                rq = [0] * g.P
                for m in range(k, A.mt):
                    q = g.prow(m + A.it0)
                    if q == A.myrow and own_col:
                        pack.add(A.offset(m, k), A.tile_rows(m), kb, b_off=rq[q])
                    unpack[q].add(rq[q], A.tile_rows(m), kb, b_off=(m - k) * mb)
                    rq[q] += A.tile_rows(m)
                st["xslots"] = [(off_q[q], rows_q[q] * kb, max(1, rows_q[q])) for q in range(g.P)]
                st["gpack"] = pack.finalize() if len(pack) else None
                st["gunpack"] = [u.finalize() if len(u) else None for u in unpack]
                st["gsent"] = rows_q[A.myrow] * kb if own_col else 0
            elif g.P > 1 and self.gbuf is not None:
                # pack my panel tiles into my slot of the gather buffer, unpack every slot into the panel
                gm, slot = self.gmax, g.P
                pack, unpack = TileBatch(), TileBatch()
                sent = 0
                for q in range(slot):
                    r = 0
                    for m in range(k, A.mt):
                        if g.prow(m + A.it0) != q:
                            continue
                        base = q * gm * kb + r
                        if q == A.myrow:
                            pack.add(A.offset(m, k), A.tile_rows(m), kb, b_off=base)
                            sent += A.tile_rows(m) * kb
                        unpack.add(base, A.tile_rows(m), kb, b_off=(m - k) * mb)
                        r += A.tile_rows(m)
                st["gpack"] = pack.finalize() if len(pack) else None
                st["gunpack"] = unpack.finalize()
                st["gsent"] = sent
            if self.pivot:
                st["plu"] = ops.PanelLU(st["pv"], mp, mp, kb, pivot=True, bw=self.panel_bw)
            else:
                # no pivoting: only the diagonal block needs the recursive LU; the rows below are
                # L21 = A21 U11^-1, one TRSM launch (no grid barrier over the tall panel)
                st["plu"] = ops.PanelLU(st["pv"], mp, kb, kb, pivot=False)
                if mp > kb:
                    tb = TileBatch()
                    for r in range(kb, mp, mb):
                        tb.add(0, min(mb, mp - r), kb, b_off=r)
                    st["l21"] = tb.finalize()
            if g.P > 1 and own_col:
                # percol mode: my panel rows, contiguous (ld = Ml), and their global row indices
                lg, lu_ = TileBatch(), TileBatch()
                grow, r = [], 0
                mine = [m for m in range(k, A.mt) if A.row_is_local(m)]
                Ml = sum(A.tile_rows(m) for m in mine)
                for m in mine:
                    lg.add(A.offset(m, k), A.tile_rows(m), kb, b_off=r)
                    lu_.add(r, A.tile_rows(m), kb, b_off=(m - k) * mb)
                    grow += list(range(m * mb, m * mb + A.tile_rows(m)))
                    r += A.tile_rows(m)
                st["Ml"] = Ml
                st["lgather"], st["lunpack"] = lg.finalize(), lu_.finalize()
                st["grow"] = grow
        trail = [n for n in range(k + 1, A.nt) if A.col_is_local(n)]
        st["trail"] = trail
        lcols = self.lcols
        st["jl"] = bisect.bisect_left(lcols, k)                       # local columns left of the panel
        st["jk"] = 1 if A.col_is_local(k) else 0                        # the panel column itself (rewritten by back)
        st["jn"] = 1 if (k + 1 < A.nt and A.col_is_local(k + 1)) else 0   # the next panel's column
        parts = {"": trail, "_n": trail[:st["jn"]], "_r": trail[st["jn"]:]}
        if trail and A.row_is_local(k):
            for sfx, cols in parts.items():
                if cols:
                    tb = TileBatch()
                    for n in cols:
                        tb.add(0, kb, A.tile_cols(n), b_off=A.offset(k, n))
                    st["trsm" + sfx] = tb.finalize()
        if trail and k + 1 < A.mt:
            uoff, c = {}, 0
            for n in trail:
                uoff[n] = c * kb
                c += A.tile_cols(n)
            st["ulen"] = c * kb
            st["ulen_n"] = (A.tile_cols(k + 1) * kb) if st["jn"] else 0   # the next column's U leads the buffer
            if A.row_is_local(k):
                for sfx, cols in parts.items():
                    if cols:
                        tb = TileBatch()
                        for n in cols:
                            tb.add(A.offset(k, n), kb, A.tile_cols(n), b_off=uoff[n])
                        st["upack" + sfx] = tb.finalize()
            rows = [m for m in range(k + 1, A.mt) if A.row_is_local(m)]
            if rows:
                nxt, rest = GemmBatch(), GemmBatch()
                for n in trail:
                    for m in rows:
                        (nxt if n == k + 1 else rest).add(A.offset(m, n), A.tile_rows(m), A.tile_cols(n),
                                                          [(lay[m], uoff[n], kb)])
                st["gemm_next"] = nxt.finalize() if len(nxt) else None
                st["gemm_rest"] = rest.finalize() if len(rest) else None
        # xmode: the rest columns in chunks -- (first, end) local column index, columns, U range; per chunk its TRSM,
        # U pack and update batch
        rest_cols = trail[st["jn"]:]
        j0r = st["jl"] + st["jk"] + st["jn"]
        bnd = [round(c * len(rest_cols) / self.nch) for c in range(self.nch + 1)]
        st["chunks"] = []
        for c in range(self.nch):
            cols = rest_cols[bnd[c]:bnd[c + 1]]
            ch = {"j0": j0r + bnd[c], "j1": j0r + bnd[c + 1], "cols": cols}
            if cols and "ulen" in st:
                ch["ulo"] = uoff[cols[0]]
                ch["uhi"] = uoff[cols[-1]] + A.tile_cols(cols[-1]) * kb
                if A.row_is_local(k):
                    tb, up = TileBatch(), TileBatch()
                    for n in cols:
                        tb.add(0, kb, A.tile_cols(n), b_off=A.offset(k, n))
                        up.add(A.offset(k, n), kb, A.tile_cols(n), b_off=uoff[n])
                    ch["trsm"], ch["upack"] = tb.finalize(), up.finalize()
                rows = [m for m in range(k + 1, A.mt) if A.row_is_local(m)]
                if rows:
                    gb = GemmBatch()
                    for n in cols:
                        for m in rows:
                            gb.add(A.offset(m, n), A.tile_rows(m), A.tile_cols(n), [(lay[m], uoff[n], kb)])
                    ch["gemm"] = gb.finalize()
            elif cols and A.row_is_local(k):
                tb = TileBatch()
                for n in cols:
                    tb.add(0, kb, A.tile_cols(n), b_off=A.offset(k, n))
                ch["trsm"] = tb.finalize()
            st["chunks"].append(ch)
        return st

    def step(self, k):
        """The whole step in order (no look-ahead)."""
        self.panel(k)
        if self.xmode:
            self.swap_next(k)
            self.next(k)
            for c in range(len(self.plan[k]["chunks"])):
                self.swap_rest(k, c)
                self.rest_chunk(k, c)
            self.swap_left(k)
            return
        self.swap(k)
        self.next(k)
        self.rest(k)

    def panel(self, k):
        A, ctx = self.A, self.ctx
        g = A.grid
        st = self.plan[k]
        kb, r0, mp, kmin = st["kb"], st["r0"], st["mp"], st["kmin"]
        pc = g.pcol(k + A.jt0)
        pv = st["pv"][: st["pld"] * kb]
        # --- gather the panel in its process column (each process row sends only its own tiles)
        if A.col_is_local(k) and self.dist:
            self._panel_dist(k)
        elif A.col_is_local(k) and self.percol:
            self._panel_percol(k)
        elif self.gxp2p:
            self._panel_gx(k)
            return self._panel_tail(k, pv)
        elif A.col_is_local(k):
            if g.P > 1:
                gv = self.gbuf[: g.P * self.gmax * kb].view(g.P, self.gmax * kb)
                if st["gpack"] is not None:
                    ops.geadd(0, N_, 1.0, A.data, A.ld, 0.0, self.gbuf, self.gmax, st["gpack"], copy=True)
                comm.allgather_inplace(gv, A.myrow, ctx.col_group)
                ops.geadd(0, N_, 1.0, self.gbuf, self.gmax, 0.0, pv, mp, st["gunpack"], copy=True)
                self.bytes_panel[k] = st["gsent"]
            elif "gather" in st:
                ops.geadd(0, N_, 1.0, A.data, A.ld, 0.0, pv, mp, st["gather"], copy=True)
            st["plu"].run(self.piv_dev, self.ws, self.cnt, self.info, r0)
            if "l21" in st:
                ops.trsm(dplasmaRight, dplasmaUpper, N_, dplasmaNonUnit, 1.0, pv, mp, pv, mp, st["l21"])
        return self._panel_tail(k, pv, bcast=True)

    def _panel_tail(self, k, pv, bcast=False):
        A, ctx = self.A, self.ctx
        g = A.grid
        st = self.plan[k]
        kb, r0, kmin = st["kb"], st["r0"], st["kmin"]
        pc = g.pcol(k + A.jt0)
        # --- factored panel + pivots along process rows
        if bcast and g.Q > 1:
            root = g.rank(A.myrow, pc)
            if "rlen" in st:        # gather mode, P > 1: only this process row's tiles travel
                rb = self.rbuf[: st["rlen"]]
                if A.col_is_local(k) and "rpack" in st:
                    ops.geadd(0, N_, 1.0, pv, st["pld"], 0.0, self.rbuf, st["rld"], st["rpack"], copy=True)
                comm.bcast(rb, root, ctx.row_group)
                if not A.col_is_local(k) and "runpack" in st:
                    ops.geadd(0, N_, 1.0, self.rbuf, st["rld"], 0.0, pv, st["pld"], st["runpack"], copy=True)
            else:
                comm.bcast(pv, root, ctx.row_group)
            if self.pivot:
                comm.bcast(self.piv_dev, root, ctx.row_group)
        if not self.pivot:
            return
        self.ipiv_all[r0: r0 + kmin].copy_(self.piv_dev[:kmin] + (r0 + 1))
        if self.tmp is not None:   # net moves of this step's interchanges (lists double-buffered by parity)
            par = k & 1
            ops.piv_moves(self.piv_dev, kmin, self.mdst[par], self.msrc[par], self.mcnt[par], mrel=self.A.m - r0,
                          info=self.info)
            if self.xmode:
                ops.rows_xord(self.mdst[par], self.msrc[par], self.mcnt[par], r0, A.mb, self.prow_t, A.myrow, g.P,
                              A.nb, self.xo[par], self.info)

    def _panel_gx(self, k):
        """Gather-mode panel on P x Q with point-to-point transfers of the exact per-step slots.  The ranks of the
        panel's process column exchange their tiles; with RNF the ranks of the next panel's column receive every
        slot too, and all of them factor the panel redundantly (identical pivots).  The other ranks of each process
        row get that row's tiles of the factored panel and the pivots from the panel's column, point to point on the
        row communicator."""
        A, ctx = self.A, self.ctx
        g = A.grid
        st = self.plan[k]
        kb = st["kb"]
        pv = st["pv"]
        kc = g.pcol(k + A.jt0)
        kc1 = g.pcol(k + 1 + A.jt0) if (self.rnf and k + 1 < A.nt) else None
        in_k = A.col_is_local(k)
        in_k1 = kc1 is not None and A.mycol == kc1 and not in_k
        if st.get("fac"):
            sl = st["xslots"]
            gb = self.gbuf
            if in_k and st["gpack"] is not None:
                o, n, ldq = sl[A.myrow]
                ops.geadd(0, N_, 1.0, A.data, A.ld, 0.0, gb[o:], ldq, st["gpack"], copy=True)
            sends, recvs = [], []
            if in_k:
                o, n, _ = sl[A.myrow]
                dst = [g.rank(q, kc) for q in range(g.P) if q != A.myrow]
                if kc1 is not None:
                    dst += [g.rank(q, kc1) for q in range(g.P)]
                sends = [(gb[o:o + n], d) for d in dst] if n else []
                recvs = [(gb[sl[q][0]:sl[q][0] + sl[q][1]], g.rank(q, kc)) for q in range(g.P)
                         if q != A.myrow and sl[q][1]]
            else:
                recvs = [(gb[sl[q][0]:sl[q][0] + sl[q][1]], g.rank(q, kc)) for q in range(g.P) if sl[q][1]]
            comm.p2p(sends, recvs, group=self.g_next)
            for q in range(g.P):   # every slot into the full panel (mine too: the pack read it from A)
                if st["gunpack"][q] is not None:
                    ops.geadd(0, N_, 1.0, gb[sl[q][0]:], sl[q][2], 0.0, pv, st["mp"], st["gunpack"][q], copy=True)
            self.bytes_panel[k] = st["gsent"]
            st["plu"].run(self.piv_dev, self.ws, self.cnt, self.info, st["r0"])
            if in_k:   # (LSEND task: PANEL(k+1) re-fills piv_dev before LSEND(k) may run)
                self.piv_send[k & 1].copy_(self.piv_dev)
        if g.Q > 1:
            others = [c for c in range(g.Q) if c != kc and c != kc1]
            mine = g.rank(A.myrow, kc)
            if in_k and others and not self.lsend_task:
                self._lsend(k)
            elif not in_k and not st.get("fac"):
                recvs = [(self.piv_dev, mine)]
                if "rlen" in st and st["rlen"]:
                    recvs.append((self.rbuf[: st["rlen"]], mine))
                comm.p2p((), recvs, group=ctx.row_group)
                if "rlen" in st and st["rlen"]:
                    ops.geadd(0, N_, 1.0, self.rbuf, st["rld"], 0.0, pv, st["pld"], st["runpack"], copy=True)

    def _lsend(self, k):
        """The factored panel's rows of my process row and the pivots, from the panel's column to the other ranks of
        the row (point to point on the row communicator).  With look-ahead a task of its own (LSEND, own stream):
        neither the panel owner's next steps nor its trailing updates wait for these transfers."""
        A, ctx = self.A, self.ctx
        g = A.grid
        if not (self.gxp2p and g.Q > 1 and A.col_is_local(k)):
            return
        st = self.plan[k]
        kc = g.pcol(k + A.jt0)
        kc1 = g.pcol(k + 1 + A.jt0) if (self.rnf and k + 1 < A.nt) else None
        others = [c for c in range(g.Q) if c != kc and c != kc1]
        if not others:
            return
        sends = [(self.piv_send[k & 1], g.rank(A.myrow, c)) for c in others]
        if "rlen" in st and st["rlen"]:
            rb = self.rbuf_send[k & 1] if self.rbuf_send is not None else self.rbuf
            ops.geadd(0, N_, 1.0, st["pv"], st["pld"], 0.0, rb, st["rld"], st["rpack"], copy=True)
            sends += [(rb[: st["rlen"]], g.rank(A.myrow, c)) for c in others]
        comm.p2p(sends, (), group=ctx.row_group)

    def _panel_dist(self, k):
        """Distributed partial pivoting of panel k on the GPUs of its process column (see panel_mode):
        the diagonal tile is replicated down the column, then every rank factors its (T + own rows)
        buffer with the exchange kernel; the pivots come out identical on every rank."""
        A, ctx = self.A, self.ctx
        g = A.grid
        st = self.plan[k]
        kb, tr, pld = st["kb"], st["tr"], st["pld"]
        pv = st["pv"]
        ops.geadd(0, N_, 1.0, A.data, A.ld, 0.0, pv, pld, st["gather"], copy=True)
        tb = self.tbuf[: tr * kb]
        if "tpack" in st:
            ops.geadd(0, N_, 1.0, A.data, A.ld, 0.0, tb, tr, st["tpack"], copy=True)
        comm.bcast(tb, g.rank(g.prow(k + A.it0), A.mycol), ctx.col_group)
        if "tunpack" in st:
            ops.geadd(0, N_, 1.0, tb, tr, 0.0, pv, pld, st["tunpack"], copy=True)
        st["plu"].run(self.piv_dev, self.dws, self.cnt, self.info, st["r0"], self.xc)
        self.bytes_panel[k] = self.bytes_panel_plan[k]

    def close(self):
        """Drop this factorisation's reference to the (cached, re-used) exchange buffers."""
        self.xc = None

    def _panel_percol(self, k):
        """Distributed partial pivoting of panel k inside its process column (see panel_mode)."""
        A, ctx = self.A, self.ctx
        g = A.grid
        st = self.plan[k]
        kb, r0, kmin, Ml = st["kb"], st["r0"], st["kmin"], st["Ml"]
        W = 2 + 2 * kb
        lp = self.lpbuf
        if Ml:
            ops.geadd(0, N_, 1.0, A.data, A.ld, 0.0, lp, Ml, st["lgather"], copy=True)
        L = torch.as_strided(lp, (Ml, kb), (1, max(Ml, 1)), 0)
        grow = st["grow"]
        where = {gr: i for i, gr in enumerate(grow)}
        diag_owner = A.row_is_local(k)
        diag_rank = g.prow(k + A.it0)
        xb = self.xbuf[: g.P * W].view(g.P, W)
        cplx = A.dtype.is_complex
        crit = (lambda x: x.real.abs() + x.imag.abs()) if cplx else (lambda x: x.abs())  # noqa: E731 (i?amax)
        piv = [0] * kmin
        bad = 0
        for j in range(kmin):
            lo = j if diag_owner else 0          # rows still eligible: global index >= r0 + j
            mine = xb[A.myrow]
            mine.zero_()
            mine[0] = -1.0
            if Ml > lo:
                c = crit(L[lo:, j])
                i = int(torch.argmax(c).item())   # first maximum, as i?amax
                mine[0] = c[i]
                mine[1] = float(grow[lo + i])
                mine[2:2 + kb] = L[lo + i, :]
            if diag_owner:
                mine[2 + kb:] = L[j, :]
            comm.allgather_inplace(xb, A.myrow, ctx.col_group)
            hv = xb[:, :2].real.cpu().tolist() if cplx else xb[:, :2].cpu().tolist()
            best = max(range(g.P), key=lambda q: (hv[q][0], -hv[q][1]))
            pg = int(hv[best][1])
            u = xb[best, 2:2 + kb].clone()
            piv[j] = pg - r0
            if pg != r0 + j:
                d = xb[diag_rank, 2 + kb:]
                if pg in where:
                    L[where[pg], :] = d
                if diag_owner:
                    L[j, :] = u
            b0 = j + 1 if diag_owner else 0
            if u[j] == 0:
                bad = bad or (r0 + j + 1)
                continue
            if Ml > b0:
                L[b0:, j] /= u[j]
                if j + 1 < kb:
                    L[b0:, j + 1:] -= torch.outer(L[b0:, j], u[j + 1:])
        self.bytes_panel[k] = kmin * W
        if bad and int(self.info.item()) == 0:
            self.info.fill_(bad)
        if Ml:
            ops.geadd(0, N_, 1.0, lp, Ml, 0.0, st["pv"], st["mp"], st["lunpack"], copy=True)
        self.piv_dev[:kmin] = torch.tensor(piv, dtype=torch.int32, device=self.piv_dev.device)

    def swap(self, k):
        A, ctx = self.A, self.ctx
        g = A.grid
        st = self.plan[k]
        kb, r0, mp, pld = st["kb"], st["r0"], st["mp"], st["pld"]
        pv = st["pv"][: pld * kb]
        # --- row interchanges on every local column (the panel column is rewritten below)
        if not self.pivot:
            pass
        elif self.percol and self.tmp is not None:
            # pivots are on the host in this mode: only the rows that cross process rows travel,
            # between the two process rows involved (one all-to-all of exact sizes per column group)
            piv = self.piv_dev[: st["kmin"]].cpu().numpy()
            perm = _perm_from_swaps(piv, mp)
            moved = np.nonzero(perm != np.arange(mp))[0]
            if len(moved):
                _permute_rows_2d(ctx, A, r0 + moved, r0 + perm[moved], self.lcols)
        elif self.tmp is not None:
            par = k & 1
            mdst, msrc, mcnt = self.mdst[par], self.msrc[par], self.mcnt[par]
            ldb = 2 * A.nb
            nl = self.nleft[k] if (self.side is not None or self.trailing_only) else 0
            cur = torch.cuda.current_stream() if self.side is not None else None
            if cur is not None and self.ev_side[par] is not None:
                cur.wait_event(self.ev_side[par])      # step k-2's side moves have read these lists
            if nl and self.side is not None:
                ev = torch.cuda.Event()
                ev.record(cur)                           # lists ready, left columns final (back(k-1))
                with torch.cuda.stream(self.side):
                    self.side.wait_event(ev)
                    cl, nc = self.coloff[:nl], self.ncols[:nl]
                    ops.rows_move(True, A.data, A.ld, A.mb, r0, self.rowoff, cl, nc, A.nb, msrc, mcnt, ldb,
                                  self.tmp_l, ldb, self.info)
                    ops.rows_move(False, A.data, A.ld, A.mb, r0, self.rowoff, cl, nc, A.nb, mdst, mcnt, ldb,
                                  self.tmp_l, ldb, self.info)
                    self.ev_side[par] = torch.cuda.Event()
                    self.ev_side[par].record(self.side)
            cr, nr = self.coloff[nl:], self.ncols[nl:]
            if g.P == 1 and self.inplace_moves and ldb <= 1024:
                # one process: in-place permutation, no staging round trip through HBM
                ops.rows_permute(A.data, A.ld, A.mb, r0, self.rowoff, cr, nr, A.nb, mdst, msrc, mcnt, ldb, self.info)
            else:
                ops.rows_move(True, A.data, A.ld, A.mb, r0, self.rowoff, cr, nr, A.nb, msrc, mcnt, ldb, self.tmp,
                              ldb, self.info)
                if g.P > 1:
                    comm.allreduce(self.tmp, group=ctx.col_group)
                ops.rows_move(False, A.data, A.ld, A.mb, r0, self.rowoff, cr, nr, A.nb, mdst, mcnt, ldb, self.tmp,
                              ldb, self.info)
            if cur is not None and k == self.kt - 1:
                for e in self.ev_side:                   # join: the factorisation ends with L final
                    if e is not None:
                        cur.wait_event(e)
                self.ev_side = [None, None]
        if "back" in st:
            ops.geadd(0, N_, 1.0, pv, pld, 0.0, A.data, A.ld, st["back"], copy=True)
        # --- U block row where it lives, then down the process column
        if not st["trail"]:
            return
        if "trsm" in st:
            ops.trsm(dplasmaLeft, dplasmaLower, N_, dplasmaUnit, 1.0, pv, pld, A.data, A.ld, st["trsm"])
        if "ulen" not in st:
            return
        ub = self.ubuf
        if "upack" in st:
            ops.geadd(0, N_, 1.0, A.data, A.ld, 0.0, ub, kb, st["upack"], copy=True)
        if g.P > 1:
            comm.bcast(ub[: st["ulen"]], g.rank(g.prow(k + A.it0), A.mycol), ctx.col_group)

    # ---- P > 1 interchanges, point to point (xmode) ------------------------------------------------------
    def _xswap(self, k, j0, j1, tmp, key, group):
        """Step k's net row moves on the local tile columns lcols[j0:j1]: my source rows are staged (gather), the
        ones whose destination lies on another process row go into that row's send buffer at their class ordinal
        (rows_xord / rows_xcopy), one grouped point-to-point exchange with the other process rows of my column
        (fixed NB-row buffers: a class never holds more than NB moves), the arriving rows are unpacked into their
        staging slots and every slot is scattered to its local destination row."""
        if j1 <= j0:
            return
        A = self.A
        g = A.grid
        st = self.plan[k]
        par = k & 1
        nb = A.nb
        ldb = 2 * nb
        W = (j1 - j0) * nb
        xb = self.xb[key]
        rows = tmp is not None
        if rows:
            cr, nr = self.coloff[j0:j1], self.ncols[j0:j1]
            ops.rows_move(True, A.data, A.ld, A.mb, st["r0"], self.rowoff, cr, nr, nb, self.msrc[par], self.mcnt[par],
                          ldb, tmp, ldb, self.info)
            ops.rows_xcopy(True, tmp, ldb, W, self.xo[par], self.mcnt[par], ldb, xb["sp"], nb)
        sends = [(xb["send"][q][: nb * W], g.rank(q, A.mycol)) for q in self.xpeers]
        recvs = [(xb["recv"][q][: nb * W], g.rank(q, A.mycol)) for q in self.xpeers]
        comm.p2p(sends, recvs, group=group)
        if rows:
            ops.rows_xcopy(False, tmp, ldb, W, self.xo[par], self.mcnt[par], ldb, xb["rp"], nb)
            ops.rows_move(False, A.data, A.ld, A.mb, st["r0"], self.rowoff, cr, nr, nb, self.mdst[par], self.mcnt[par],
                          ldb, tmp, ldb, self.info)

    def _u_bcast(self, k, sfx, lo, hi, group):
        """U block row part [lo, hi) of ubuf (packed where row k lives) down the process column, point to point
        from the diagonal process row on ``group``."""
        A, st = self.A, self.plan[k]
        if hi <= lo:
            return
        g = A.grid
        ubuf = self.ubufs[k & 1]
        ub = ubuf[lo:hi]
        pk = st.get("upack" + sfx) if isinstance(sfx, str) else sfx.get("upack")
        if pk is not None:
            ops.geadd(0, N_, 1.0, A.data, A.ld, 0.0, ubuf, st["kb"], pk, copy=True)
        root_p = g.prow(k + A.it0)
        if A.myrow == root_p:
            comm.p2p([(ub, g.rank(q, A.mycol)) for q in range(g.P) if q != root_p], (), group=group)
        else:
            comm.p2p((), [(ub, g.rank(root_p, A.mycol))], group=group)

    def swap_next(self, k):
        """The next panel's column (k + 1) only: interchanges, panel write-back, its U block and broadcast -- the
        critical path of the look-ahead (panel stream)."""
        A, st = self.A, self.plan[k]
        j0 = st["jl"] + st["jk"]
        self._xswap(k, j0, j0 + st["jn"], self.tmp_n, "next", self.g_next)
        if "back" in st:
            ops.geadd(0, N_, 1.0, st["pv"], st["pld"], 0.0, A.data, A.ld, st["back"], copy=True)
        if "trsm_n" in st:
            ops.trsm(dplasmaLeft, dplasmaLower, N_, dplasmaUnit, 1.0, st["pv"], st["pld"], A.data, A.ld, st["trsm_n"])
        if "ulen" in st:
            self._u_bcast(k, "_n", 0, st["ulen_n"], self.g_next)

    def swap_rest(self, k, c):
        """Chunk c of the later trailing columns: interchanges, U blocks, broadcast (exchange stream)."""
        A, st = self.A, self.plan[k]
        ch = st["chunks"][c]
        self._xswap(k, ch["j0"], ch["j1"], self.tmp, "rest", self.g_rest)
        if "trsm" in ch:
            ops.trsm(dplasmaLeft, dplasmaLower, N_, dplasmaUnit, 1.0, st["pv"], st["pld"], A.data, A.ld, ch["trsm"])
        if "ulo" in ch:
            self._u_bcast(k, ch, ch["ulo"], ch["uhi"], self.g_rest)

    def rest_chunk(self, k, c):
        st = self.plan[k]
        gb = st["chunks"][c].get("gemm")
        if gb is not None:
            ops.gemm(N_, N_, -1.0, st["pv"], st["pld"], self.ubufs[k & 1], st["kb"], 1.0, self.A.data, self.A.ld, gb)

    def swap_left(self, k):
        """The already factored columns (< k): only the final L needs these moves (side stream)."""
        if self.trailing_only:
            return
        self._xswap(k, 0, self.plan[k]["jl"], getattr(self, "tmp_x", None), "left", self.g_left)

    def _update(self, k, key):
        st = self.plan[k]
        gb = st.get(key)
        if gb is not None:   # trailing update A(m, n) -= L(m, k) U(k, n)
            ops.gemm(N_, N_, -1.0, st["pv"], st["pld"], self.ubufs[k & 1], st["kb"], 1.0, self.A.data, self.A.ld, gb)

    def next(self, k):
        self._update(k, "gemm_next")

    def rest(self, k):
        # DPLASMA_LU_REST_CAP=n (look-ahead): the bulk update as a grid-stride GEMM of at most n workgroups, so
        # the next panel's persistent kernel finds room on every CU beside it instead of waiting for drains
        cap = int(os.environ.get("DPLASMA_LU_REST_CAP", "0")) if self.lookahead else 0
        if cap > 0:
            with ops.gemm_wg_cap(cap):
                self._update(k, "gemm_rest")
        else:
            self._update(k, "gemm_rest")

    def left_all(self):
        """The deferred left interchanges (defer_left): column n's rows below its diagonal block take the composition
        of steps n+1 .. kt-1's interchanges.  One host read of the pivots, after the last step."""
        if not self.defer_left or self.kt < 2:
            return
        from ..runtime.dag import _lib_rt
        A = self.A
        mb = A.mb
        ip = self.ipiv_all[: min(A.m, A.n)].cpu().numpy()
        src, off = _lib_rt().piv_compose_left(ip, A.m, mb, self.kt)
        srcd = torch.from_numpy(src).to(self.dev)
        buf = self.__dict__.get("_lbuf")
        need = max(1, (A.m - mb) * A.nb)
        if buf is None or buf.numel() < need:
            buf = self._lbuf = torch.empty(need, dtype=A.dtype, device=self.dev)
        for j, n in enumerate(self.lcols):
            if n >= self.kt - 1:
                break
            s0 = (n + 1) * mb
            cnt = A.m - s0
            o = int(off[n])
            ops.rows_perm_col(A.data, A.ld, mb, self.rowoff, self.coloff_h[j], A.tile_cols(n), srcd[o:o + cnt], s0, cnt,
                              buf, self.info)

    def add_tasks(self, tp, tag):
        """PANEL/SWAP/NEXT/REST tasks of every step; with look-ahead PANEL(k+1) overlaps REST(k)."""
        if not self.lookahead:
            prev = None
            for k in range(self.kt):
                prev = tp.task(f"{tag}({k})", "update", (lambda k=k: self.step(k)), [prev])
            if self.defer_left:
                tp.task("LEFTALL", "update", self.left_all, [prev])
            return
        nxt = rest = None
        if self.xmode:
            # PANEL(k+1) waits for NEXT(k) only; SWAPN(k+1) for REST(k) (column k+2 carries step k's update);
            # LEFT(k) on the low-priority side stream after PANEL(k) (move lists; panel k-1 written back before
            # PANEL(k) by SWAPN(k-1) on the panel stream) -- PANEL(k+2) re-fills step k's lists, so it waits for LEFT(k)
            # REST(k) runs in column chunks on the update stream; SWAPR(k) chunk c (exchange stream) waits only for
            # the chunks of REST(k-1) that updated its columns, so its transfers overlap the update of the others;
            # SWAPN(k) waits for the chunk of REST(k-1) that updated column k+1.  PANEL(k) re-fills step k-2's panel
            # buffer, move lists and U buffer: it waits for all of REST(k-2) and LEFT(k-2).
            lefts, rest_of, col_chunk, lsends = {}, {}, {}, {}
            xs = "xch" if self.dev.type == "cuda" else "update"
            for k in range(self.kt):
                st = self.plan[k]
                t_p = tp.task(f"PANEL({k})", "panel", (lambda k=k: self.panel(k)),
                              [nxt, lefts.get(k - 2)] + rest_of.get(k - 2, []) + [lsends.get(k - 2)], prio=3)
                if self.lsend_task:
                    ls_s = "lsend" if self.dev.type == "cuda" else "update"
                    lsends[k] = tp.task(f"LSEND({k})", ls_s, (lambda k=k: self._lsend(k)), [t_p], prio=3)
                t_n = tp.task(f"SWAPN({k})", "panel", (lambda k=k: self.swap_next(k)),
                              [t_p, col_chunk.get((k - 1, k + 1))], prio=3)
                nxt = tp.task(f"NEXT({k})", "panel", (lambda k=k: self.next(k)), [t_n], prio=2)
                rest_of[k] = []
                for c, ch in enumerate(st["chunks"]):
                    if not ch["cols"]:
                        continue
                    dr = [t_p] + sorted({col_chunk[(k - 1, n)] for n in ch["cols"] if (k - 1, n) in col_chunk})
                    t_x = tp.task(f"SWAPR{c}({k})", xs, (lambda k=k, c=c: self.swap_rest(k, c)), dr, prio=2)
                    t_r = tp.task(f"REST{c}({k})", "update", (lambda k=k, c=c: self.rest_chunk(k, c)), [t_x], prio=1)
                    for n in ch["cols"]:
                        col_chunk[(k, n)] = t_r
                    rest_of[k].append(t_r)
                if not self.trailing_only and st["jl"] > 0:
                    lefts[k] = tp.task(f"LEFT({k})", "aux", (lambda k=k: self.swap_left(k)),
                                       [t_p, lefts.get(k - 1)], prio=0)
            tail = ([t for t in lefts.values()] + [t for v in rest_of.values() for t in v[-1:]] + [nxt]
                    + [t for t in lsends.values()][-1:])
            tp.task("JOIN", "update", (lambda: None), tail, prio=0)   # the factorisation ends with L final
            return
        for k in range(self.kt):
            t_p = tp.task(f"PANEL({k})", "panel", (lambda k=k: self.panel(k)), [nxt], prio=3)
            t_s = tp.task(f"SWAP({k})", "update", (lambda k=k: self.swap(k)), [t_p, rest], prio=2)
            nxt = tp.task(f"NEXT({k})", "panel", (lambda k=k: self.next(k)), [t_s], prio=2)
            rest = tp.task(f"REST({k})", "update", (lambda k=k: self.rest(k)), [t_s], prio=1)
        if self.defer_left:
            tp.task("LEFTALL", "update", self.left_all, [nxt, rest], prio=0)


def _permute_rows_2d(ctx, A, dst_rows, src_rows, coltiles):
    """A[dst_rows[i], tiles] := A_old[src_rows[i], tiles] (global element rows of the view) on a P x Q grid.

    Rows live on process rows ``prow(row // mb)``; for one process column all
    ranks agree on the move lists (they depend only on the replicated pivots),
    so moves across process rows are ONE all-to-all inside the process-column
    group (RCCL p2p), local moves are two row-gather launches.  All sources are
    read before any destination is written (the moves form a permutation)."""
    if len(dst_rows) == 0:
        return
    mb, nb = A.mb, A.nb
    g, myrow = A.grid, A.myrow
    P = g.P
    prow = lambda r: g.prow(r // mb + A.it0)  # noqa: E731
    coltiles = list(coltiles)
    dst_p = np.array([prow(int(r)) for r in dst_rows])
    src_p = np.array([prow(int(r)) for r in src_rows])
    local = np.nonzero((dst_p == myrow) & (src_p == myrow))[0]
    sends = [np.nonzero((src_p == myrow) & (dst_p == q))[0] for q in range(P)]
    recvs = [np.nonzero((dst_p == myrow) & (src_p == q))[0] for q in range(P)]
    for q in range(P):
        if q == myrow:
            sends[q] = recvs[q] = np.zeros(0, dtype=np.int64)
    cross = P > 1 and any(((src_p != dst_p)).tolist())
    nct = len(coltiles)

    def off(r, n):
        return A.offset(r // mb, n) + r % mb

    # element offset of (row r, tile column n) = off(r, n0) + colpart(n) - colpart(n0): both storages are
    # affine in the local tile column index
    from ..constants import STORAGE_TILE
    cw = np.array([A.tile_cols(n) for n in coltiles], dtype=np.int64)
    jl = np.array([A.lcol[n + A.jt0] for n in coltiles], dtype=np.int64)
    colpart = jl * (A.llmt * A.mb * A.nb if A.storage == STORAGE_TILE else A.nb * A.ld)
    colpart = colpart - (colpart[0] if len(colpart) else 0)

    def pairs(idx_rows, slot0, to_buf):
        """(row_gather pairs per width group): slot j holds one tile row of nb elements (vectorised over
        rows x tile columns)."""
        rp = np.array([off(int(r), coltiles[0]) for r in idx_rows], dtype=np.int64)
        j = np.arange(len(rp), dtype=np.int64)
        slots = (slot0 + j[:, None] * nct + np.arange(nct, dtype=np.int64)[None, :]) * nb
        offs = rp[:, None] + colpart[None, :]
        out = {}
        for w in np.unique(cw).tolist():
            sel = np.broadcast_to(cw[None, :] == w, offs.shape)
            a, b = (slots[sel], offs[sel]) if to_buf else (offs[sel], slots[sel])
            pr = np.zeros(len(a), dtype=ops.ROW_PAIR)
            pr[pr.dtype.names[0]], pr[pr.dtype.names[1]] = a, b
            out[int(w)] = pr
        return out

    dev, dt = A.device, A.dtype
    tmp = torch.empty(max(1, len(local) * nct) * nb, dtype=dt, device=dev)
    if len(local) and nct:
        for w, pr in pairs(src_rows[local], 0, True).items():
            ops.row_gather(tmp, A.data, pr, w, 1, A.ld)
    if cross:
        scount = [len(s) * nct * nb for s in sends]
        rcount = [len(r) * nct * nb for r in recvs]
        sbuf = torch.empty(sum(scount), dtype=dt, device=dev)
        rbuf = torch.empty(sum(rcount), dtype=dt, device=dev)
        slot = 0
        for q in range(P):
            if len(sends[q]) and nct:
                for w, pr in pairs(src_rows[sends[q]], slot, True).items():
                    ops.row_gather(sbuf, A.data, pr, w, 1, A.ld)
            slot += len(sends[q]) * nct
        dist.all_to_all_single(rbuf, sbuf, output_split_sizes=rcount, input_split_sizes=scount,
                               group=ctx.col_group)
    if len(local) and nct:
        for w, pr in pairs(dst_rows[local], 0, False).items():
            ops.row_gather(A.data, tmp, pr, w, A.ld, 1)
    if cross:
        slot = 0
        for q in range(P):
            if len(recvs[q]) and nct:
                for w, pr in pairs(dst_rows[recvs[q]], slot, False).items():
                    ops.row_gather(A.data, rbuf, pr, w, A.ld, 1)
            slot += len(recvs[q]) * nct


def _reduce_info(info: torch.Tensor) -> int:
    """Combine the per-rank LU info: a negative code on ANY rank (-1000: a persistent panel
    kernel's grid barrier timed out, the factorisation is corrupt) raises; otherwise the smallest
    positive singular-pivot index wins (LAPACK reports the first zero pivot)."""
    v = info.to(torch.int64)
    neg = torch.where(v < 0, v, torch.zeros_like(v))
    comm.allreduce(neg, op=torch.distributed.ReduceOp.MIN)
    if int(neg.item()) < 0:
        code = int(neg.item())
        if code == ops.BAD_PIVOT:
            raise RuntimeError(f"getrf: an out-of-range pivot reached the row interchanges on some rank (info={code}):"
                               " no row was moved by that step, the factorisation is invalid")
        raise RuntimeError(f"getrf: panel kernel failed on some rank (info={code}): the grid of "
                           "the persistent panel kernel was not co-resident")
    big = torch.iinfo(torch.int64).max
    pos = torch.where(v > 0, v, torch.full_like(v, big))
    comm.allreduce(pos, op=torch.distributed.ReduceOp.MIN)
    r = int(pos.item())
    return 0 if r == big else r


def getrf_ptgpanel_New(ctx, A, IPIV, info_out=None):
    """Partial-pivoting LU on any P x Q grid (dplasma_zgetrf_ptgpanel_New).

    IPIV: P x min(M,N) int32 with 1 x NB tiles (one replicated row per process
    row, tests/testing_zgetrf_ptgpanel.c:55-58) or the 1-D ``ipiv_descriptor``."""
    tp = Taskpool("getrf_ptgpanel", ctx)
    tp.flops = flops(A.prec, "getrf", A.m, A.n)
    info = torch.zeros(1, dtype=torch.int32, device=A.device)
    st = _GetrfDev(ctx, A, info)
    st.add_tasks(tp, "getrf_ptg")
    tp._state = st

    def _done():
        for (m, n) in IPIV.local_tiles():
            c0 = n * IPIV.nb
            IPIV.tile(m, n).copy_(st.ipiv_all[c0: c0 + IPIV.tile_cols(n)].view(1, -1).to(IPIV.device))
        r = _reduce_info(info)
        if info_out is not None:
            info_out[0] = r
        return r
    tp.on_complete(_done)
    tp.on_destruct(st.close)
    tp.ipiv_all = st.ipiv_all
    return tp.finish_build()


def getrf_ptgpanel(ctx, A, IPIV):
    return getrf_ptgpanel_New(ctx, A, IPIV).execute(ctx)


def ptgpanel_ipiv_descriptor(ctx, A, name="IPIV") -> TiledMatrix:
    """P x min(M,N) int32, 1 x NB tiles: one replicated pivot row per process row."""
    k = min(A.m, A.n)
    return TiledMatrix(torch.int32, 1, A.nb, A.grid.P, k, P=A.grid.P, Q=A.grid.Q, rank=ctx.rank, device=A.device,
                       name=name)


def getrf_1d_New(ctx, A, IPIV, info_out=None):
    if ctx.world > 1 and A.P != 1:
        return getrf_ptgpanel_New(ctx, A, IPIV, info_out)  # 2-D grid: the P x Q variant
    tp = Taskpool("getrf_1d", ctx)
    tp.flops = flops(A.prec, "getrf", A.m, A.n)
    info = torch.zeros(1, dtype=torch.int32, device=A.device)
    st = _GetrfDev(ctx, A, info)
    st.add_tasks(tp, "getrf1d")
    tp._state = st

    def _done():
        # IPIV descriptor: every tile owner writes its piece (values are replicated)
        for (m, n) in IPIV.local_tiles():
            c0 = n * IPIV.nb
            IPIV.tile(m, n).copy_(st.ipiv_all[c0: c0 + IPIV.tile_cols(n)].view(1, -1).to(IPIV.device))
        r = _reduce_info(info)
        if info_out is not None:
            info_out[0] = r
        return r
    tp.on_complete(_done)
    tp.on_destruct(st.close)
    tp.ipiv_all = st.ipiv_all
    return tp.finish_build()


def getrf_1d(ctx, A, IPIV):
    return getrf_1d_New(ctx, A, IPIV).execute(ctx)


getrf = getrf_1d


# ----------------------------------------------------------------------------- LASWP / GETRS / GESV
def _gather_ipiv(ctx, IPIV) -> np.ndarray:
    k = IPIV.n
    full = torch.zeros(k, dtype=torch.int32, device=IPIV.device)
    for (m, n) in IPIV.local_tiles():
        if m != 0:  # ptgpanel IPIV: one replicated row per process row
            continue
        c0 = n * IPIV.nb
        full[c0: c0 + IPIV.tile_cols(n)] = IPIV.tile(m, n).view(-1)
    if ctx.world > 1:
        comm.allreduce(full)
    return full.cpu().numpy()


def laswp(ctx, A, IPIV, inc=1):
    """Apply the row interchanges of IPIV (1-based, sequential) to A, forward (inc>0) or backward.

    Any P x Q grid: rows crossing process rows move with one all-to-all per
    process column (_permute_rows_2d)."""
    piv = _gather_ipiv(ctx, IPIV) - 1
    # an out-of-range pivot (i <= piv[i] < m violated) moves nothing and is reported, never wrapped around
    if len(piv) > A.m or np.any(piv < np.arange(len(piv))) or np.any(piv >= A.m):
        return ops.BAD_PIVOT
    perm = np.arange(A.m)
    seq = range(len(piv)) if inc > 0 else range(len(piv) - 1, -1, -1)
    for i in seq:
        p = int(piv[i])
        if p != i:
            perm[i], perm[p] = perm[p], perm[i]
    moved = np.nonzero(perm != np.arange(A.m))[0]
    cols = [n for n in range(A.nt) if A.col_is_local(n)]
    _permute_rows_2d(ctx, A, moved, perm[moved], cols)
    if A.device.type == "cuda":
        torch.cuda.synchronize(A.device)
    return 0


def trsmpl_ptgpanel(ctx, A, IPIV, B):
    """B := L^-1 P B with the getrf_ptgpanel factors (dplasma_ztrsmpl_ptgpanel)."""
    rc = laswp(ctx, B, IPIV, 1)
    if rc:
        return rc
    blas3.trsm(ctx, dplasmaLeft, dplasmaLower, N_, dplasmaUnit, 1.0, A, B)
    return 0


def gerfs(ctx, A, LU, IPIV, B, X, iters=2):
    """Iterative refinement X += (LU)^-1 (B - A X) (dplasma_zgerfs role)."""
    from . import aux
    from .gemm import gemm
    R = B.like(name="R")
    for _ in range(iters):
        aux.lacpy(ctx, 123, B, R)  # dplasmaUpperLower
        gemm(ctx, N_, N_, -1.0, A, X, 1.0, R)
        getrs(ctx, N_, LU, IPIV, R)
        aux.geadd(ctx, N_, 1.0, R, 1.0, X)
    return 0


def getrs(ctx, trans, A, IPIV, B):
    """Solve op(A) X = B with the getrf_1d factorization (A = P L U)."""
    if trans == N_:
        rc = laswp(ctx, B, IPIV, 1)
        if rc:
            return rc
        blas3.trsm(ctx, dplasmaLeft, dplasmaLower, N_, dplasmaUnit, 1.0, A, B)
        blas3.trsm(ctx, dplasmaLeft, dplasmaUpper, N_, dplasmaNonUnit, 1.0, A, B)
    else:
        piv = _gather_ipiv(ctx, IPIV) - 1
        if len(piv) > B.m or np.any(piv < np.arange(len(piv))) or np.any(piv >= B.m):
            return ops.BAD_PIVOT   # checked before the solves: B is left unchanged
        blas3.trsm(ctx, dplasmaLeft, dplasmaUpper, trans, dplasmaNonUnit, 1.0, A, B)
        blas3.trsm(ctx, dplasmaLeft, dplasmaLower, trans, dplasmaUnit, 1.0, A, B)
        return laswp(ctx, B, IPIV, -1)
    return 0


def gesv_1d(ctx, A, IPIV, B):
    info = getrf_1d(ctx, A, IPIV)
    if info != 0:
        return info
    return getrs(ctx, N_, A, IPIV, B)


def getrs_nopiv(ctx, trans, A, B):
    if trans == N_:
        blas3.trsm(ctx, dplasmaLeft, dplasmaLower, N_, dplasmaUnit, 1.0, A, B)
        blas3.trsm(ctx, dplasmaLeft, dplasmaUpper, N_, dplasmaNonUnit, 1.0, A, B)
    else:
        blas3.trsm(ctx, dplasmaLeft, dplasmaUpper, trans, dplasmaNonUnit, 1.0, A, B)
        blas3.trsm(ctx, dplasmaLeft, dplasmaLower, trans, dplasmaUnit, 1.0, A, B)
    return 0


def gesv_nopiv(ctx, A, B):
    info = getrf_nopiv(ctx, A)
    if info != 0:
        return info
    return getrs_nopiv(ctx, N_, A, B)
