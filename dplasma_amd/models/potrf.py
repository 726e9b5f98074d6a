"""Cholesky factorization (POTRF) -- the headline algorithm.

Reference: ``src/zpotrf_L.jdf`` / ``zpotrf_U.jdf`` (task classes potrf_zpotrf(k)
:93, potrf_ztrsm(m,k) :194, potrf_zherk(k,m) :306, potrf_zgemm(m,n,k) :407)
and ``src/zpotrf_wrapper.c:175-336`` (New / blocking / Destruct, info
all-reduce).

MI355X design (not a translation of the JDF):

* The factorisation is compiled (``potrf_New``) into a short program of
  coarse tasks per step k, right-looking with look-ahead 1:

    panel stream  : POTRF(k) -> bcast diag tile down the owner column ->
                    TRSM of the local panel tiles (ONE batched launch) ->
                    pack + row broadcast + column all-gather of the panel
    update stream : UPDCOL(k)  trailing update of tile column k+1 (one launch)
                    UPDREST(k) trailing update of every other local tile
                               (one launch of the MFMA GEMM engine over all
                               local (m, n) tiles, diagonal tiles masked lower)

  POTRF(k+1) depends only on UPDCOL(k), so the k+1 panel (on the
  high-priority stream) overlaps UPDREST(k) -- the critical-path/lookahead
  structure the reference obtains with priorities (zpotrf_L.jdf:58-69).
* Tiles stay resident in HBM; the panel travels once per step over RCCL/xGMI:
  the owner column broadcasts its pieces along process rows and every
  process column all-gathers them, so each rank ends with the full panel in
  a double-buffered contiguous slab (buffer k%2).
* Single rank: no copies at all -- the panel is read in place.
"""
from __future__ import annotations

import torch

from ..constants import (STORAGE_TILE, dplasmaConjTrans, dplasmaLeft, dplasmaLower, dplasmaNoTrans, dplasmaNonUnit,
                         dplasmaRight, dplasmaUpper)
from ..ops import tile_ops as ops
from ..ops.batch import MASK_LOWER, MASK_UPPER, GemmBatch, TileBatch
from ..parallel import comm
from ..runtime import Taskpool
from ..utils.flops import flops


class _Panel:
    """Where the step-k panel tiles live for the update: (base tensor, ld, offset(i))."""

    def __init__(self, base, ld, off_fn):
        self.base, self.ld, self.off = base, ld, off_fn


def potrf_New(ctx, uplo: int, A, info_out=None) -> Taskpool:
    """Build the Cholesky taskpool for the ``uplo`` triangle of square matrix A."""
    if uplo not in (dplasmaLower, dplasmaUpper):
        raise ValueError("potrf: illegal uplo")
    if A.m != A.n or A.mb != A.nb:
        raise ValueError("potrf: A must be square with square tiles")
    lower = uplo == dplasmaLower
    tp = Taskpool("potrf", ctx)
    tp.flops = flops(A.prec, "potrf", A.n)
    nt = A.nt
    dev = A.device
    nbe = A.mb * A.nb
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    tp.info = info
    distributed = ctx.world > 1
    P, Q = A.P, A.Q
    myrow, mycol = A.myrow, A.mycol

    # "panel coordinate": lower -> tile (i, k); upper -> tile (k, i)
    def tcoord(i, k):
        return (i, k) if lower else (k, i)

    def owner_of_panel_line(i):  # process row (lower) / col (upper) index of panel tile i
        return A.grid.prow(i + A.it0) if lower else A.grid.pcol(i + A.jt0)

    my_line = myrow if lower else mycol          # my index along the panel distribution axis
    nlines = P if lower else Q
    line_group = ctx.col_group if lower else ctx.row_group   # ranks sharing my column (lower)
    cross_group = ctx.row_group if lower else ctx.col_group  # ranks sharing my row (lower)

    def panel_owner_cross(k):  # process col (lower) / row (upper) that owns panel k
        return A.grid.pcol(k + A.jt0) if lower else A.grid.prow(k + A.it0)

    my_cross = mycol if lower else myrow

    # distributed panel buffers: G[2][nlines][maxcnt][nbe]
    if distributed:
        maxcnt = 0
        for k in range(nt):
            cnt = [0] * nlines
            for i in range(k + 1, nt):
                cnt[owner_of_panel_line(i)] += 1
            maxcnt = max(maxcnt, max(cnt) if cnt else 0)
        maxcnt = max(maxcnt, 1)
        G = torch.zeros(2, nlines, maxcnt, nbe, dtype=A.dtype, device=dev)
        dbuf = torch.zeros(nbe, dtype=A.dtype, device=dev)
        tp._buffers = (G, dbuf)

    tri_mask = MASK_LOWER if lower else MASK_UPPER
    prev_col = None   # task id of UPDCOL(k-1)
    last_upd = {}     # k -> last update-stream task of step k (guards panel buffer reuse)
    prev_panel = None
    for k in range(nt):
        kb = A.tile_rows(k)
        dk = tcoord(k, k)
        own_diag = A.is_local(*dk)
        in_panel_cross = (panel_owner_cross(k) == my_cross)
        # ---------------- POTRF(k)
        t_potrf = None
        if own_diag:
            off = A.offset(*dk)

            def f_potrf(off=off, kb=kb, k=k):
                ops.potrf_tile(uplo, A.data, off, kb, A.ld, info, k * A.mb)
            t_potrf = tp.task(f"POTRF({k})", "panel", f_potrf, [prev_col], prio=3)
        # ---------------- local panel tiles (i > k) of my process row/col
        mine = [i for i in range(k + 1, nt) if in_panel_cross and owner_of_panel_line(i) == my_line]
        # ---------------- diag tile to the panel owners (column for lower) and TRSM
        t_trsm = None
        if in_panel_cross:
            if distributed and nlines > 1:
                src = A.grid.rank(*((owner_of_panel_line(k), panel_owner_cross(k)) if lower
                                    else (panel_owner_cross(k), owner_of_panel_line(k))))
                dk_off = A.offset(*dk) if own_diag else None

                def f_dbcast(dk_off=dk_off, src=src, kb=kb):
                    if dk_off is not None:
                        dv = torch.as_strided(dbuf, (kb, kb), (1, A.mb), 0)
                        dv.copy_(torch.as_strided(A.data, (kb, kb), (1, A.ld), dk_off))
                    comm.bcast(dbuf, src, line_group)
                t_db = tp.task(f"DBCAST({k})", "panel", f_dbcast, [t_potrf, prev_col], prio=3)
                tri_base, tri_ld, tri_off = dbuf, A.mb, 0
            else:
                t_db = t_potrf
                tri_base, tri_ld, tri_off = A.data, A.ld, A.offset(*dk)
            if mine:
                tb = TileBatch()
                for i in mine:
                    c = tcoord(i, k)
                    tb.add(tri_off, A.tile_rows(c[0]), A.tile_cols(c[1]), b_off=A.offset(*c))
                tb.finalize()
                side = dplasmaRight if lower else dplasmaLeft

                def f_trsm(tb=tb, tri_base=tri_base, tri_ld=tri_ld, side=side):
                    ops.trsm(side, uplo, dplasmaConjTrans, dplasmaNonUnit, 1.0, tri_base, tri_ld, A.data, A.ld, tb)
                t_trsm = tp.task(f"TRSM({k})", "panel", f_trsm, [t_db, prev_col], prio=2)
        # ---------------- panel distribution
        if k == nt - 1:
            break
        if distributed:
            par = k % 2
            lines_cnt = [0] * nlines
            idx_in_line = {}
            for i in range(k + 1, nt):
                ln = owner_of_panel_line(i)
                idx_in_line[i] = lines_cnt[ln]
                lines_cnt[ln] += 1
            my_cnt = lines_cnt[my_line]
            pack = None
            if in_panel_cross and mine:
                pb = TileBatch()
                for j, i in enumerate(mine):
                    c = tcoord(i, k)
                    pb.add(A.offset(*c), A.tile_rows(c[0]), A.tile_cols(c[1]),
                           b_off=((par * nlines + my_line) * maxcnt + j) * nbe)
                pack = pb.finalize()
            root = A.grid.rank(*((my_line, panel_owner_cross(k)) if lower else (panel_owner_cross(k), my_line)))

            def f_comm(pack=pack, par=par, my_cnt=my_cnt, root=root):
                if pack is not None:
                    # local slab -> G[par][my_line] (ld = mb)
                    ops.geadd(0, dplasmaNoTrans, 1.0, A.data, A.ld, 0.0, G, A.mb, pack, copy=True)
                if my_cnt > 0 and cross_group is not None:
                    comm.bcast(G[par, my_line, :my_cnt], root, cross_group)
                if line_group is not None:
                    comm.allgather_inplace(G[par], my_line, line_group)
            deps = [t_trsm, prev_col, prev_panel, last_upd.get(k - 2)]
            t_panel = tp.task(f"PANEL_COMM({k})", "panel", f_comm, deps, prio=2)

            def poff(i, par=par, idx_in_line=idx_in_line):
                return ((par * nlines + owner_of_panel_line(i)) * maxcnt + idx_in_line[i]) * nbe
            panel = _Panel(G, A.mb, poff)
        else:
            t_panel = t_trsm if t_trsm is not None else t_potrf
            panel = _Panel(A.data, A.ld, lambda i, k=k: A.offset(*tcoord(i, k)))
        prev_panel = t_panel
        # ---------------- trailing update: tiles (m, n) with k < n <= m (lower)
        col_b, rest_b = GemmBatch(), GemmBatch()
        for n_ in range(k + 1, nt):
            for m_ in range(n_, nt):
                c = (m_, n_) if lower else (n_, m_)
                if not A.is_local(*c):
                    continue
                kp = [(panel.off(c[0] if lower else c[0]), panel.off(c[1]), kb)]
                b = col_b if n_ == k + 1 else rest_b
                b.add(A.offset(*c), A.tile_rows(c[0]), A.tile_cols(c[1]), kp, tri_mask if m_ == n_ else 0)
        col_b.finalize()
        rest_b.finalize()
        tA, tB = (dplasmaNoTrans, dplasmaConjTrans) if lower else (dplasmaConjTrans, dplasmaNoTrans)

        def f_upd(batch, panel=panel, tA=tA, tB=tB):
            ops.gemm(tA, tB, -1.0, panel.base, panel.ld, panel.base, panel.ld, 1.0, A.data, A.ld, batch)
        t_col = None
        if len(col_b):
            t_col = tp.task(f"UPDCOL({k})", "update", lambda b=col_b, f=f_upd: f(b), [t_panel], prio=2)
            last_upd[k] = t_col
        if len(rest_b):
            last_upd[k] = tp.task(f"UPDREST({k})", "update", lambda b=rest_b, f=f_upd: f(b), [t_panel], prio=1)
        prev_col = t_col

    def _done():
        v = info.clone()
        if distributed:
            comm.allreduce(v, op=torch.distributed.ReduceOp.MAX)
        r = int(v.item())
        if info_out is not None:
            info_out[0] = r
        return r
    tp.on_complete(_done)
    return tp.finish_build()


def potrf(ctx, uplo: int, A) -> int:
    """Blocking Cholesky: returns info (0 = success, >0 = order of the failing leading minor)."""
    tp = potrf_New(ctx, uplo, A)
    return tp.execute(ctx)


def potrf_Destruct(tp: Taskpool):
    tp.destruct()
