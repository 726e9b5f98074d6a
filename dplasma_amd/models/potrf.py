"""Cholesky factorization (POTRF) -- the headline algorithm.

Reference: ``src/zpotrf_L.jdf`` / ``zpotrf_U.jdf`` (task classes potrf_zpotrf(k)
:93, potrf_ztrsm(m,k) :194, potrf_zherk(k,m) :306, potrf_zgemm(m,n,k) :407)
and ``src/zpotrf_wrapper.c:175-336`` (New / blocking / Destruct, info
all-reduce).

MI355X design (not a translation of the JDF):

* The factorisation is compiled (``potrf_New``) into a short program of
  coarse tasks, right-looking over blocks of D panels (deferred updates):

    panel stream  : POTRF(k) -> bcast diag tile down the owner column ->
                    TRSM of the local panel tiles (ONE batched launch) ->
                    pack + row broadcast + column all-gather of the panel ->
                    NEAR(k): panel k updates the rest of its block
    update stream : NEXT(b)  block b's D panels update block b+1 (k = D*NB)
                    REST(b)  ... and every local tile beyond it (one launch of
                             the MFMA GEMM engine, diagonal tiles masked)

  Block b+1's panels depend only on NEXT(b), so they (high-priority stream)
  overlap REST(b) -- the critical-path/lookahead structure the reference
  obtains with priorities (zpotrf_L.jdf:58-69).
* Tiles stay resident in HBM; the panel travels once per step over RCCL/xGMI:
  the owner column broadcasts its pieces along process rows (each rank needs
  every panel tile of its own rows), then inside each process column only the
  tiles that column needs as the second GEMM operand are all-gathered -- a
  rank receives (nt-k)/P + (nt-k)(P-1)/(PQ) tiles per panel, not (nt-k).
* Single rank: no copies at all -- the panel is read in place.
"""
from __future__ import annotations

import os

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


POTRF_DEFER = 4            # panels aggregated per deferred trailing update (k = 4*NB)
POTRF_DEFER_MIN_TILES = 24 # below this many trailing tile-columns: plain look-ahead-1 (D = 1)
# Diagonal-tile kernel: "single" = one-workgroup left-looking kernel, "blocked" = 128-wide
# right-looking steps over several workgroups.  Measured on MI355X (profiles/r1_potrf_tile_kernels.txt):
# 577 vs 625 us for a 512 tile in isolation, but DPOTRF 32k (the per-GPU share of 64k on 8 GPUs)
# 53.0 vs 56.7 TF/s -- its extra launches contend with the bulk update -- so "single" everywhere;
# "auto" = blocked when distributed.
POTRF_TILE = "single"
POTRF_LOOKAHEAD = 1
POTRF_TRSM = "rb"   # "fused": the diagonal owner factors its tile and solves its panel strips in one launch
# CUs kept free of the bulk trailing updates (REST / NEXT2 / REST2 run as capped grid-stride GEMM
# launches of 2 x (CUs - reserve) workgroups, ops.gemm_wg_cap): the panel chain's kernels find idle
# CUs instead of waiting for GEMM workgroups to retire.  (single process, distributed)
POTRF_RESERVE = (0, 0)
# one GPU process: "stream" (the stream-program engine below), "dtr" (the device task runtime,
# models/potrf_dtr.py) or "auto" (dtr for POTRF_DTR_MIN_N <= N < POTRF_DTR_MAX_N when it supports the
# operand).  Measured (profiles/r4_dtr_colorder.txt, r4_b16): 32k dtr 63-64 vs stream 61-62 TF/s; 64k dtr
# 68.4-69.3 vs stream 69.4-70.1 (the stream engine's D = 2 deferred updates run the GEMMs at their
# large-k rate, which the DTR's 128 x 128 x 512 update tasks do not reach); 16k dtr 38 vs 47.
# Round 5: the DTR runs one workgroup per CU (two per CU gave an intermittent wrong factor under stress --
# round 6 found and fixed the cause, an inline-asm store, profiles/r6_dtr_coresidency_rootcause.txt; one per CU
# stays the default because it is faster) and push-schedules its tasks by bottom level (profiles/r5_dtr_queue.txt):
# 16k 48.8 / 32k 62.0 / 64k 65.2 TF/s against the stream engine's 46.0 / 59.5-61.2 / 67.0-69.2 -> "auto" takes
# the DTR below 48k.
POTRF_ENGINE = "auto"
POTRF_DTR_MIN_N = 12288
POTRF_DTR_MAX_N = 49152


def _defer_depth(nt_left: int, D: int, min_tiles: int) -> int:
    return D if nt_left >= min_tiles else 1


def potrf_New(ctx, uplo: int, A, info_out=None, defer: int = None) -> Taskpool:
    """Build the Cholesky taskpool for the ``uplo`` triangle of square matrix A.

    Blocked right-looking schedule with deferred (aggregated) trailing updates:
    panels are processed in blocks of D tile-columns (``defer``, default
    ``POTRF_DEFER``; D = 1 once fewer than ``POTRF_DEFER_MIN_TILES`` columns
    remain).  Inside a block each panel k updates the rest of its own block at
    once (NEAR(k), panel stream, critical path).  The D panels of a block then
    update the next block (NEXT(b), critical path of the next block) and every
    column beyond it (REST(b), which overlaps the next block's panels) in single
    launches whose k-runs are D*NB long: the MFMA engine runs at its large-k rate
    (74 vs 70 TF/s at k=512 on MI355X) and every trailing tile is read and
    written once per block instead of once per panel.
    """
    if uplo not in (dplasmaLower, dplasmaUpper):
        raise ValueError("potrf: illegal uplo")
    if A.m != A.n or A.mb != A.nb:
        raise ValueError("potrf: A must be square with square tiles")
    # memory-capped variant: a host-resident matrix on a GPU context, or an explicit arena cap
    # (reference: the device memory manager's bounded block pool, tests/Testings.cmake:147)
    if ctx.world == 1 and ((ctx.is_gpu and A.data.device.type == "cpu")
                           or ctx.info.get_int("DPLASMA:GPU:number_of_blocks", 0) > 0):
        from .potrf_ooc import potrf_ooc_New
        return potrf_ooc_New(ctx, uplo, A)
    # one process, lower, fp64, NB = 512: the whole factorisation as one persistent launch of the device
    # task runtime (panel work prioritised inside the bulk update's workgroups, models/potrf_dtr.py)
    eng = os.environ.get("DPLASMA_POTRF_ENGINE", POTRF_ENGINE)
    if eng in ("dtr", "auto"):
        from . import potrf_dtr
        # auto: the device task runtime in its measured window (below it the panel chain dominates and the
        # stream engine's register-resident panel solve is faster; above it the stream engine's deferred
        # large-k updates win: profiles/r4_dtr_*.txt)
        win = (int(os.environ.get("DPLASMA_POTRF_DTR_MIN_N", POTRF_DTR_MIN_N)) <= A.n
               < int(os.environ.get("DPLASMA_POTRF_DTR_MAX_N", POTRF_DTR_MAX_N)))
        if potrf_dtr.supported(ctx, uplo, A) and (eng == "dtr" or win):
            return potrf_dtr.potrf_dtr_New(ctx, uplo, A, info_out)
        if eng == "dtr" and ctx.world > 1:
            # one rank of a P x Q grid: the distributed device task runtime (models/potrf_dtr_dist.py)
            from . import potrf_dtr_dist
            if potrf_dtr_dist.supported(ctx, uplo, A):
                return potrf_dtr_dist.potrf_dtr_dist_New(ctx, uplo, A, info_out)
        if eng == "dtr":
            raise ValueError("DPLASMA_POTRF_ENGINE=dtr: needs lower, fp64, NB = 512, N % 512 == 0 (one GPU process, or a "
                             "P x Q grid of <= 8 GPU processes with TILE storage)")
    if (ctx.world > 1 or getattr(ctx, "loopback", False)) and os.environ.get("DPLASMA_POTRF_DIST", "p2p") != "collective":
        # distributed: point-to-point dataflow panel transport (models/potrf_dist.py);
        # DPLASMA_POTRF_DIST=collective keeps the row-broadcast + column-all-gather schedule below
        from .potrf_dist import potrf_dist_New
        return potrf_dist_New(ctx, uplo, A, info_out)
    # Upper on one process: factor A^T (A^H) with the lower schedule (transposed copies in and out,
    # ops.copy_transpose, overlapped with the factorisation) instead of the upper tile kernels, whose
    # strips are strided columns of U (16k: native upper 40.1 vs lower 46.7 TF/s,
    # profiles/r3_potrf_upper_via_lower.txt).  DPLASMA_POTRF_UPPER=native keeps the upper kernels.
    up_mode = os.environ.get("DPLASMA_POTRF_UPPER", "auto")
    via_lower = uplo == dplasmaUpper and ctx.world == 1 and (up_mode == "via_lower" or (ctx.is_gpu and up_mode == "auto"))
    if via_lower:
        uplo = dplasmaLower
    lower = uplo == dplasmaLower
    tp = Taskpool("potrf", ctx)
    t_in = t_in1 = None
    if via_lower:
        # the lower schedule factors a workspace copy W = A^T (A^H) of the upper triangle; each block of
        # columns of W goes back into A's upper triangle once factored (A's strictly lower part is never
        # touched).  One read + one write of the triangle each way, overlapped with the factorisation.
        cj = A.dtype.is_complex
        A_user = A
        A = A_user.like(name="W")

        def xpose(cols, back=False):
            xb, db = TileBatch(), TileBatch()
            for j in cols:
                for i in range(j, A.mt):
                    if back:
                        (db if i == j else xb).add(A.offset(i, j), A.tile_rows(i), A.tile_cols(j),
                                                   b_off=A_user.offset(j, i))
                    else:
                        xb.add(A_user.offset(j, i), A_user.tile_rows(j), A_user.tile_cols(i), b_off=A.offset(i, j))
            xb.finalize()
            db.finalize()
            src, dst = (A, A_user) if back else (A_user, A)

            def f(xb=xb, db=db):
                ops.copy_transpose(src.data, src.ld, dst.data, dst.ld, xb, conj=cj)
                ops.copy_transpose(src.data, src.ld, dst.data, dst.ld, db, conj=cj, upper_only=True)
            return f
        xposed_out = set()
    # diagonal tiles on the CU-reserved stream when DPLASMA_DIAG_CUS is set (context._reserve_cus)
    diag_stream = "diag" if "diag" in getattr(ctx, "streams", {}) else "panel"
    # the panel TRSM joins the diagonal tile on the CU-reserved stream (DPLASMA_POTRF_DIAG_TRSM=0: on
    # the shared panel stream): both are latency-bound chains that slow 7-28x beside GEMM waves
    # (profiles/r2_potrf16k_timeline.txt)
    trsm_stream = diag_stream if os.environ.get("DPLASMA_POTRF_DIAG_TRSM", "1") == "1" else "panel"
    upd_stream = "potrf_update" if "potrf_update" in getattr(ctx, "streams", {}) else "update"
    # PRI_CHANGE ({S,D,C,Z}POTRF env, reference zpotrf_wrapper.c:201-203): the last PRI_CHANGE
    # panels issue their critical-path tasks at normal priority (update stream) instead of the
    # high-priority panel stream; 0 (default) keeps every panel on the panel stream
    from ..utils.aux import get_priority_limit
    pri_change = get_priority_limit("POTRF", A)

    def pstream(k, default):
        return upd_stream if (pri_change > 0 and k >= A.nt - pri_change) else default
    tp.flops = flops(A.prec, "potrf", A.n)
    nt = A.nt
    dev = A.device
    nbe = A.mb * A.nb
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    tp.info = info
    distributed = ctx.world > 1
    P, Q = A.P, A.Q
    myrow, mycol = A.myrow, A.mycol
    if defer is None:
        defer = int(os.environ.get("DPLASMA_POTRF_DEFER", POTRF_DEFER))
    D = max(1, int(defer))
    min_tiles = int(os.environ.get("DPLASMA_POTRF_DEFER_MIN_TILES", POTRF_DEFER_MIN_TILES))
    # look-ahead depth: 1 -- NEXT(b) follows the whole bulk update REST(b-1) on the update stream;
    # 2 -- REST(b) is split into NEXT2(b) (the columns of block b+2) and REST2(b) (beyond), NEXT(b)
    # moves to the panel stream and needs only NEXT2(b-1): the bulk update gets two blocks of slack
    la = int(os.environ.get("DPLASMA_POTRF_LOOKAHEAD", POTRF_LOOKAHEAD))
    if la not in (1, 2):
        raise ValueError("DPLASMA_POTRF_LOOKAHEAD must be 1 or 2")
    nslab = 1 + la          # panel slabs in flight (distributed): block b+nslab reuses block b's
    # panel TRSM: "rb" (register-resident strips on the tile kernel's inverted 32-blocks) or "gemm"
    # (inverse of the diagonal tile + one MFMA GEMM launch: bulk-efficient beside the trailing GEMM)
    trsm_kind = os.environ.get("DPLASMA_POTRF_TRSM", POTRF_TRSM)
    if trsm_kind not in ("rb", "gemm", "fused"):
        raise ValueError("DPLASMA_POTRF_TRSM must be rb, fused or gemm")
    tile_kind = os.environ.get("DPLASMA_POTRF_TILE", POTRF_TILE)
    if tile_kind not in ("auto", "single", "blocked"):
        raise ValueError(f"DPLASMA_POTRF_TILE={tile_kind!r}: expected auto, single or blocked")
    # auto: the single-workgroup tile kernel only where nothing better exists -- fp64 uses the dataflow
    # kernel (use_rb below); distributed runs and the other precisions take nb-wide MFMA sub-steps
    # (a complex 512 tile on one workgroup is ~10 ms: zpotrf 32k 33.0 -> 47.2 TF/s with sub-steps,
    # profiles/r2_zpotrf_tile.txt)
    potrf_diag = ops.potrf_tile_blocked if tile_kind == "blocked" or (
        tile_kind == "auto" and (distributed or A.dtype != torch.float64)) else ops.potrf_tile

    # block partition of the tile columns
    blocks = []
    c = 0
    while c < nt:
        d = _defer_depth(nt - c, D, min_tiles)
        blocks.append((c, min(nt, c + d)))
        c += d

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

    def cross_of(i):  # process col (lower) / row (upper) of panel tile i's "other" index
        return A.grid.pcol(i + A.jt0) if lower else A.grid.prow(i + A.it0)

    # Distributed panel buffers, one flat tensor GX; per (block parity, panel in block) a slab of
    #   G [nlines][maxcnt][nbe]: every line's panel tiles (my line arrives by the row broadcast)
    #   X [nlines][maxsub][nbe]: of every line, only the tiles my process column/row needs as the
    #                            second GEMM operand (cross_of(i) == my_cross), all-gathered
    # so each rank receives (nt-k)/P + (nt-k)(P-1)/(PQ) tiles per panel instead of (nt-k).
    if distributed:
        maxcnt = maxsub = 1
        for k in range(nt):
            cnt, sub = [0] * nlines, [0] * nlines
            for i in range(k + 1, nt):
                ln = owner_of_panel_line(i)
                cnt[ln] += 1
                if cross_of(i) == my_cross:
                    sub[ln] += 1
            maxcnt = max(maxcnt, max(cnt) if cnt else 0)
            maxsub = max(maxsub, max(sub) if sub else 0)
        SG, SX = nlines * maxcnt * nbe, nlines * maxsub * nbe
        slab = SG + SX
        GX = torch.zeros(nslab * D * slab, dtype=A.dtype, device=dev)
        dbuf = torch.zeros(nbe, dtype=A.dtype, device=dev)
        dpack = torch.zeros(A.mb * (A.mb + 1) // 2, dtype=A.dtype, device=dev)
        tp._buffers = (GX, dbuf, dpack)

    # fp64 tiles <= 512 on the GPU: dataflow tile POTRF + register-resident panel TRSM sharing the
    # inverted diagonal 32-blocks (csrc/kernels/potrf_rb.hip); zbufs alternate with k's parity
    use_rb = ops.rb_ok(A.data, A.mb) and A.mb == A.nb
    if use_rb:
        zsz = ops.rb_zbuf_size()
        zbufs = torch.empty(2 * zsz, dtype=torch.float64, device=dev)
        tp._zbufs = zbufs
    tri_mask = MASK_LOWER if lower else MASK_UPPER
    tA, tB = (dplasmaNoTrans, dplasmaConjTrans) if lower else (dplasmaConjTrans, dplasmaNoTrans)
    panels = {}       # k -> _Panel (where panel k's tiles live for the updates)

    def add_update(batch, ks, ncols):
        """Trailing tiles (m, n), n in ncols, m >= n (lower), updated by the panels ks."""
        batch.rec = []    # (trailing tile, panel tile rows, panels) for the recursive incarnation
        for n_ in ncols:
            for m_ in range(n_, nt):
                cc = (m_, n_) if lower else (n_, m_)
                if not A.is_local(*cc):
                    continue
                batch.rec.append((cc, m_, n_, list(ks)))
                # lower: C(m,n) -= L(m,k) L(n,k)^H ; upper: C(n,m) -= U(k,n)^H U(k,m)
                kp = [(panels[k].off(cc[0]), panels[k].off(cc[1]), A.tile_rows(k)) for k in ks]
                batch.add(A.offset(*cc), A.tile_rows(cc[0]), A.tile_cols(cc[1]), kp,
                          tri_mask if m_ == n_ else 0)
        return batch.finalize()

    def f_upd(batch, base, ld):
        if _rec_nb(tp, A) and not distributed:
            _recursive_update(tp, ctx, uplo, A, batch.rec)
            return
        ops.gemm(tA, tB, -1.0, base, ld, base, ld, 1.0, A.data, A.ld, batch)

    reserve = int(os.environ.get("DPLASMA_POTRF_RESERVE", POTRF_RESERVE[1 if distributed else 0]))
    bulk_cap = 0
    if reserve > 0 and ctx.is_gpu:
        ncu = torch.cuda.get_device_properties(dev).multi_processor_count
        bulk_cap = 2 * max(8, ncu - reserve)      # k_gemm_full holds 2 workgroups per CU

    def f_bulk(batch, base, ld):
        with ops.gemm_wg_cap(bulk_cap):
            f_upd(batch, base, ld)

    if via_lower:
        # the first block's columns on the critical stream, the rest beside its panels (bulk stream);
        # each block's columns go back as soon as its last reader is done (TRANSPOSE_OUT(b) below)
        t_in = tp.task("TRANSPOSE_IN(0)", "panel", xpose(range(blocks[0][0], blocks[0][1])), [], prio=3, comm=False)
        if blocks[0][1] < nt:
            t_in1 = tp.task("TRANSPOSE_IN(1)", upd_stream, xpose(range(blocks[0][1], nt)), [], prio=1, comm=False)
    gate = t_in        # task the next POTRF must follow (NEAR(k-1) or NEXT(b-1))
    last_upd = {}      # block -> last update-stream task reading its panels
    nxt2_of, rest_of = {}, {}   # look-ahead 2: block -> NEXT2 / REST2 task (REST2: last bulk task)
    last_panel = None  # last panel-stream communication task
    for b, (c0, c1) in enumerate(blocks):
        par = b % nslab
        for k in range(c0, c1):
            kb = A.tile_rows(k)
            dk = tcoord(k, k)
            own_diag = A.is_local(*dk)
            in_panel_cross = (panel_owner_cross(k) == my_cross)
            # ---------------- POTRF(k)
            t_potrf = None
            if own_diag:
                off = A.offset(*dk)

                fused_rbp = None
                if use_rb and trsm_kind == "fused" and in_panel_cross:
                    mine_k = [i for i in range(k + 1, nt) if owner_of_panel_line(i) == my_line]
                    if mine_k:
                        fused_rbp = ops.RbPanel(uplo, [(A.offset(*tcoord(i, k)), A.tile_rows(i) if lower
                                                        else A.tile_cols(i)) for i in mine_k], A.ld)

                def f_potrf(off=off, kb=kb, k=k, dk=dk, frbp=fused_rbp,
                            mine_k=mine_k if fused_rbp is not None else ()):
                    hnb = getattr(tp, "recursive_nb", 0)
                    if hnb and hnb < kb:
                        _recursive_potrf(tp, ctx, uplo, A, dk, hnb, info, k * A.mb)
                        if frbp is not None and _rec_nb(tp, A) and not distributed:
                            _recursive_trsm(tp, ctx, uplo, A, k, mine_k)
                        elif frbp is not None:   # the sub-taskpool left no zbuf: solve the panel apart
                            zk = zbufs[(k % 2) * zsz:(k % 2 + 1) * zsz]
                            ops.trsm_rb_prep(uplo, kb, A.data, off, A.ld, zk)
                            ops.trsm_rb(uplo, kb, A.data, off, A.ld, zk, frbp, A.data, A.ld)
                    elif frbp is not None:
                        ops.potrf_trsm_rb(uplo, kb, A.data, off, A.ld, info, k * A.mb,
                                          zbufs[(k % 2) * zsz:(k % 2 + 1) * zsz], frbp, A.data, A.ld)
                    elif use_rb:
                        ops.potrf_tile(uplo, A.data, off, kb, A.ld, info, k * A.mb,
                                       zbuf=zbufs[(k % 2) * zsz:(k % 2 + 1) * zsz])
                    else:
                        potrf_diag(uplo, A.data, off, kb, A.ld, info, k * A.mb)
                t_potrf = tp.task(f"POTRF({k})", pstream(k, diag_stream), f_potrf, [gate], prio=3)
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
                        # only the factor's triangle travels (the reference's LOWER/UPPER tile shapes)
                        comm.bcast_tri(dbuf, 0, A.data if dk_off is not None else None, dk_off or 0, kb, A.ld,
                                       A.mb, lower, src, line_group, pack=dpack)
                    t_db = tp.task(f"DBCAST({k})", pstream(k, "panel"), f_dbcast, [t_potrf, gate], prio=3)
                    tri_base, tri_ld, tri_off = dbuf, A.mb, 0
                else:
                    t_db = t_potrf
                    tri_base, tri_ld, tri_off = A.data, A.ld, A.offset(*dk)
                if mine and own_diag and use_rb and trsm_kind == "fused":
                    t_trsm = t_potrf          # solved by the fused POTRF launch
                elif mine and use_rb and trsm_kind in ("rb", "fused"):
                    # row blocks of the panel tiles (lower: rows of L(i,k); upper: columns of U(k,i))
                    rbp = ops.RbPanel(uplo, [(A.offset(*tcoord(i, k)),
                                              A.tile_rows(i) if lower else A.tile_cols(i)) for i in mine], A.ld)
                    zk = zbufs[(k % 2) * zsz:(k % 2 + 1) * zsz]

                    def f_trsm(rbp=rbp, tri_base=tri_base, tri_ld=tri_ld, tri_off=tri_off, kb=kb, zk=zk,
                               own=own_diag and tri_base is A.data, k=k, mine=mine):
                        if _rec_nb(tp, A) and not distributed:
                            _recursive_trsm(tp, ctx, uplo, A, k, mine)
                            return
                        rec = 0 < getattr(tp, "recursive_nb", 0) < kb   # sub-taskpool left no zbuf
                        if rec or not own:  # the diagonal tile came by broadcast: invert its 32-blocks here
                            ops.trsm_rb_prep(uplo, kb, tri_base, tri_off, tri_ld, zk)
                        ops.trsm_rb(uplo, kb, tri_base, tri_off, tri_ld, zk, rbp, A.data, A.ld)
                    t_trsm = tp.task(f"TRSM({k})", pstream(k, trsm_stream), f_trsm, [t_db, gate], prio=2)
                elif mine:
                    tb = TileBatch()
                    for i in mine:
                        cc = tcoord(i, k)
                        tb.add(tri_off, A.tile_rows(cc[0]), A.tile_cols(cc[1]), b_off=A.offset(*cc))
                    tb.finalize()
                    side = dplasmaRight if lower else dplasmaLeft

                    def f_trsm(tb=tb, tri_base=tri_base, tri_ld=tri_ld, side=side, k=k, mine=mine):
                        if _rec_nb(tp, A) and not distributed:
                            _recursive_trsm(tp, ctx, uplo, A, k, mine)
                            return
                        ops.trsm(side, uplo, dplasmaConjTrans, dplasmaNonUnit, 1.0, tri_base, tri_ld, A.data, A.ld,
                                 tb)
                    t_trsm = tp.task(f"TRSM({k})", pstream(k, trsm_stream), f_trsm, [t_db, gate], prio=2)
            if k == nt - 1:
                break
            # ---------------- panel distribution
            if distributed:
                slot = k - c0
                o = (par * D + slot) * slab
                lines_cnt = [0] * nlines
                sub_cnt = [0] * nlines
                idx_in_line, idx_in_sub = {}, {}
                for i in range(k + 1, nt):
                    ln = owner_of_panel_line(i)
                    idx_in_line[i] = lines_cnt[ln]
                    lines_cnt[ln] += 1
                    if cross_of(i) == my_cross:
                        idx_in_sub[i] = sub_cnt[ln]
                        sub_cnt[ln] += 1
                my_cnt = lines_cnt[my_line]
                Gk = GX[o: o + SG].view(nlines, maxcnt, nbe)
                Xk = GX[o + SG: o + slab].view(nlines, maxsub, nbe)
                pack = None
                if in_panel_cross and mine:
                    pb = TileBatch()
                    for j, i in enumerate(mine):
                        cc = tcoord(i, k)
                        pb.add(A.offset(*cc), A.tile_rows(cc[0]), A.tile_cols(cc[1]),
                               b_off=o + (my_line * maxcnt + j) * nbe)
                    pack = pb.finalize()
                # my line's tiles wanted by my line_group mates -> X[my_line] (device copy)
                subpack = None
                if line_group is not None and sub_cnt[my_line]:
                    sb = TileBatch()
                    for i, t in idx_in_sub.items():
                        if owner_of_panel_line(i) == my_line:
                            sb.add(o + (my_line * maxcnt + idx_in_line[i]) * nbe, A.mb, A.nb,
                                   b_off=o + SG + (my_line * maxsub + t) * nbe)
                    subpack = sb.finalize()
                root = A.grid.rank(*((my_line, panel_owner_cross(k)) if lower else (panel_owner_cross(k), my_line)))

                def f_comm(pack=pack, subpack=subpack, Gk=Gk, Xk=Xk, my_cnt=my_cnt, root=root):
                    if pack is not None:
                        # local slab -> G[my_line] (ld = mb)
                        ops.geadd(0, dplasmaNoTrans, 1.0, A.data, A.ld, 0.0, GX, A.mb, pack, copy=True)
                    if my_cnt > 0 and cross_group is not None:
                        comm.bcast(Gk[my_line, :my_cnt], root, cross_group)
                    if line_group is not None:
                        if subpack is not None:
                            ops.geadd(0, dplasmaNoTrans, 1.0, GX, A.mb, 0.0, GX, A.mb, subpack, copy=True)
                        comm.allgather_inplace(Xk, my_line, line_group)
                # GX slab (par) is reused by block b+2: its previous readers (NEXT/REST of b-2) must be done
                t_panel = tp.task(f"PANEL_COMM({k})", pstream(k, "panel"), f_comm,
                                  [t_trsm, gate, last_panel, last_upd.get(b - nslab)], prio=2)
                last_panel = t_panel

                def poff(i, o=o, idx_in_line=idx_in_line, idx_in_sub=idx_in_sub):
                    ln = owner_of_panel_line(i)
                    if ln == my_line:
                        return o + (ln * maxcnt + idx_in_line[i]) * nbe
                    return o + SG + (ln * maxsub + idx_in_sub[i]) * nbe
                panels[k] = _Panel(GX, A.mb, poff)
            else:
                t_panel = t_trsm if t_trsm is not None else t_potrf
                panels[k] = _Panel(A.data, A.ld, lambda i, k=k: A.offset(*tcoord(i, k)))
            base, ld = panels[k].base, panels[k].ld
            # ---------------- NEAR(k): the rest of this block, right now (panel stream)
            near = add_update(GemmBatch(), [k], range(k + 1, c1))
            if len(near):
                gate = tp.task(f"NEAR({k})", pstream(k, "panel"), lambda bt=near, bs=base, l=ld: f_upd(bt, bs, l),
                               [t_panel, gate], prio=2)
            else:
                gate = t_panel if t_panel is not None else gate
        if c1 >= nt:
            break
        # ---------------- block b's panels update the next block (critical) and the rest (bulk)
        ks = list(range(c0, c1))
        n0, n1 = blocks[b + 1]
        base, ld = panels[c0].base, panels[c0].ld
        if la == 1:
            nxt = add_update(GemmBatch(), ks, range(n0, n1))
            rest = add_update(GemmBatch(), ks, range(n1, nt))
            # the previous block's bulk update touched every column beyond it: explicit WAW/RAW edge
            # (stream order alone would hold it only under program-order issue, see runtime.taskpool)
            deps = [gate, last_panel, last_upd.get(b - 1)]
            t_next = None
            if len(nxt):
                t_next = tp.task(f"NEXT({b})", upd_stream, lambda bt=nxt, bs=base, l=ld: f_upd(bt, bs, l), deps,
                                 prio=2)
                last_upd[b] = t_next
            if len(rest):
                last_upd[b] = tp.task(f"REST({b})", upd_stream, lambda bt=rest, bs=base, l=ld: f_bulk(bt, bs, l),
                                      deps, prio=1)
            if via_lower:
                tp.task(f"TRANSPOSE_OUT({b})", upd_stream, xpose(range(c0, c1), back=True),
                        [t_next, last_upd.get(b), gate, t_in1 if b == 0 else None], prio=0, comm=False)
                xposed_out.update(range(c0, c1))
            # the next block's first POTRF follows NEXT(b) (and, for this rank, the block's NEARs)
            gate = t_next if t_next is not None else gate
            continue
        n2 = blocks[b + 2][1] if b + 2 < len(blocks) else nt
        nxt = add_update(GemmBatch(), ks, range(n0, n1))
        nxt2 = add_update(GemmBatch(), ks, range(n1, n2))
        rest = add_update(GemmBatch(), ks, range(n2, nt))
        # NEXT(b): critical (panel stream); block b+1's columns were last updated by NEXT2(b-1) and,
        # before that, by REST2(b-2) (ordered before NEXT2(b-1) on the update stream)
        t_next = None
        if len(nxt):
            t_next = tp.task(f"NEXT({b})", pstream(c1, "panel"), lambda bt=nxt, bs=base, l=ld: f_upd(bt, bs, l),
                             [gate, last_panel, nxt2_of.get(b - 1), rest_of.get(b - 2)], prio=2)
        # NEXT2(b) / REST2(b): bulk (update stream); block b+2's columns and beyond were last updated
        # by REST2(b-1)
        prev_bulk = rest_of.get(b - 1)
        if len(nxt2):
            nxt2_of[b] = tp.task(f"NEXT2({b})", upd_stream, lambda bt=nxt2, bs=base, l=ld: f_bulk(bt, bs, l),
                                 [gate, last_panel, prev_bulk], prio=1)
        if len(rest):
            rest_of[b] = tp.task(f"REST2({b})", upd_stream, lambda bt=rest, bs=base, l=ld: f_bulk(bt, bs, l),
                                 [gate, last_panel, prev_bulk, nxt2_of.get(b)], prio=0)
        else:
            rest_of[b] = nxt2_of.get(b, prev_bulk)
        last_upd[b] = rest_of[b] if rest_of[b] is not None else t_next
        if via_lower:
            tp.task(f"TRANSPOSE_OUT({b})", upd_stream, xpose(range(c0, c1), back=True),
                    [t_next, nxt2_of.get(b), rest_of.get(b), gate, t_in1 if b == 0 else None], prio=0, comm=False)
            xposed_out.update(range(c0, c1))
        gate = t_next if t_next is not None else gate

    if via_lower:
        # every root task follows TRANSPOSE_IN(0), the first block's trailing updates TRANSPOSE_IN(1);
        # the columns not yet transposed back go after every task without a successor
        for t in tp.tasks:
            if t.tid in (t_in, t_in1):
                continue
            extra = []
            if not t.deps:
                extra.append(t_in)
            if t_in1 is not None and t.name in ("NEXT(0)", "REST(0)", "NEXT2(0)", "REST2(0)"):
                extra.append(t_in1)
            for d in extra:
                if d not in t.deps:
                    t.deps.append(d)
                    if tp.tasks[d].stream != t.stream:
                        tp.tasks[d].needs_event = True
        has_succ = set()
        for t in tp.tasks:
            has_succ.update(t.deps)
        sinks = [t.tid for t in tp.tasks if t.tid not in has_succ]
        left = [j for j in range(nt) if j not in xposed_out]
        if left:
            tp.task("TRANSPOSE_OUT(end)", "panel", xpose(left, back=True), sinks, prio=0, comm=False)

    def _done():
        v = info.clone()
        if distributed:
            comm.allreduce(v, op=torch.distributed.ReduceOp.MAX)
        r = int(v.item())
        if r < 0:
            # the dataflow tile kernels report a bounded-spin timeout as a negative info (-1000): an
            # execution failure, never a numerical result
            raise RuntimeError(f"potrf: tile kernel failure (info {r})")
        if info_out is not None:
            info_out[0] = r
        return r
    tp.on_complete(_done)
    return tp.finish_build()


def _recursive_potrf(tp, ctx, uplo, A, dk, hnb, info, info_base):
    """POTRF(k) as a sub-taskpool: the diagonal tile re-tiled hnb x hnb and factored by potrf_New on a
    one-process view of the context, inside the POTRF task (reference: parsec_recursivecall when
    the tile is larger than smallnb, src/zpotrf_L.jdf:148-172).  Sub-taskpools are built once per
    tile and reused; their info is folded into the parent's as base + iinfo."""
    subs = tp.__dict__.setdefault("_rec_subs", {})
    key = (dk, hnb)
    sub = subs.get(key)
    if sub is None:
        lctx = ctx.local()
        sub = subs[key] = (potrf_New(lctx, uplo, A.tile_desc(dk[0], dk[1], hnb)), lctx)
    stp, lctx = sub
    stp.info.zero_()
    stp.run(lctx)
    si = stp.info
    info.copy_(torch.where((info == 0) & (si > 0), si + info_base, info))


def _rec_nb(tp, A) -> int:
    """The recursive-incarnation tile size when dplasma_zpotrf_setrecursive asked for one smaller than
    the tiles (0: the batched tile kernels)."""
    h = int(getattr(tp, "recursive_nb", 0) or 0)
    return h if 0 < h < A.mb else 0


def _sub(tp, key, build):
    subs = tp.__dict__.setdefault("_rec_subs", {})
    sub = subs.get(key)
    if sub is None:
        sub = subs[key] = build()
    return sub


def _recursive_trsm(tp, ctx, uplo, A, k, rows):
    """TRSM(k) as sub-taskpools: every panel tile solved by trsm_New on hnb x hnb re-tilings of the tile
    and of the diagonal factor (reference: the RECURSIVE body of potrf_ztrsm, src/zpotrf_L.jdf:245-280)."""
    from .blas3 import trsm_New
    hnb = _rec_nb(tp, A)
    lower = uplo == dplasmaLower
    side = dplasmaRight if lower else dplasmaLeft
    for i in rows:
        cc = (i, k) if lower else (k, i)

        def build(cc=cc):
            lctx = ctx.local()
            return trsm_New(lctx, side, uplo, dplasmaConjTrans, dplasmaNonUnit, 1.0, A.tile_desc(k, k, hnb),
                            A.tile_desc(cc[0], cc[1], hnb)), lctx
        stp, lctx = _sub(tp, ("trsm", cc, hnb), build)
        stp.run(lctx)


def _recursive_update(tp, ctx, uplo, A, rec):
    """Trailing updates as sub-taskpools: HERK on diagonal tiles, GEMM elsewhere, on hnb x hnb re-tilings
    (reference: the RECURSIVE bodies of potrf_zherk / potrf_zgemm, src/zpotrf_L.jdf:351-390,473-520)."""
    from .blas3 import herk_New
    from .gemm import gemm_New
    hnb = _rec_nb(tp, A)
    lower = uplo == dplasmaLower
    herk_trans = dplasmaNoTrans if lower else dplasmaConjTrans
    tA, tB = (dplasmaNoTrans, dplasmaConjTrans) if lower else (dplasmaConjTrans, dplasmaNoTrans)
    for cc, m_, n_, ks in rec:
        for k in ks:
            pm = (m_, k) if lower else (k, m_)
            pn = (n_, k) if lower else (k, n_)

            def build(cc=cc, pm=pm, pn=pn, diag=(m_ == n_)):
                lctx = ctx.local()
                C = A.tile_desc(cc[0], cc[1], hnb)
                if diag:
                    return herk_New(lctx, uplo, herk_trans, -1.0, A.tile_desc(*pm, hnb), 1.0, C), lctx
                # lower: C(m,n) -= L(m,k) L(n,k)^H ; upper: C(n,m) -= U(k,n)^H U(k,m)
                a, b = (A.tile_desc(*pm, hnb), A.tile_desc(*pn, hnb)) if lower else \
                    (A.tile_desc(*pn, hnb), A.tile_desc(*pm, hnb))
                return gemm_New(lctx, tA, tB, -1.0, a, b, 1.0, C), lctx
            stp, lctx = _sub(tp, ("upd", cc, k, hnb), build)
            stp.run(lctx)


def potrf(ctx, uplo: int, A) -> int:
    """Blocking Cholesky: returns info (0 = success, >0 = order of the failing leading minor)."""
    tp = potrf_New(ctx, uplo, A)
    return tp.execute(ctx)


def potrf_Destruct(tp: Taskpool):
    tp.destruct()
