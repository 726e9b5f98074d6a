"""Distributed Cholesky (P x Q > 1 processes): dataflow panel transport.

Reference: ``src/zpotrf_L.jdf`` / ``zpotrf_U.jdf`` -- every edge from ``potrf_ztrsm(m,k)`` to a
``potrf_zherk`` / ``potrf_zgemm`` of another rank is a message sent by PaRSEC's remote-dependency
engine as soon as the TRSM finishes, with the panel tasks marked ``high_priority`` (:93,:194,:306)
and the look-ahead expressed by the priority formulas (:58-69).

MI355X design.  The schedule is the single-process one of ``models/potrf.py`` (blocks of D panels:
per panel POTRF -> panel TRSM -> NEAR; per block NEXT (the next block, critical) and REST (bulk),
optionally look-ahead 2), but the panel now travels *point to point from its producers* instead of
through a row broadcast followed by a column all-gather:

* the owner of panel tile (i, k) (a rank of process column pcol(k), lower) sends it directly to
  every rank that needs it -- the ranks of its process row (row operand: the whole piece, one
  contiguous message, the piece being packed sorted by destination column) and, in the other
  process rows, the ranks of column pcol(i) (column operand: a contiguous sub-range).  One hop, no
  relay, each pair on its own xGMI link;
* destinations are split by urgency: a rank that owns a column of the look-ahead window (the rest of
  the block and the next block: NEAR / NEXT) gets its tiles on the high-priority ``urgent``
  communicator, every other rank on a ``bulk`` communicator (``k mod DPLASMA_BULK_GROUPS``, so the
  bulk transfers of consecutive panels -- different roots -- overlap).  Each rank issues, per panel
  and communicator, ONE grouped send/recv batch (sends and receives together: no ordering deadlock);
* the receiving side waits where the data is consumed: NEAR / NEXT make the panel stream wait for the
  urgent batch, REST makes the bulk stream wait for both -- never the host, never the producer's
  stream;
* the bulk trailing updates can run on a CU-masked stream that leaves ``DPLASMA_POTRF_BULK_RESERVE``
  CUs (spread over the 8 XCDs) to the critical path and the RCCL kernels (``Context.bulk_stream``).

The diagonal tile's triangle goes to the other ranks of the panel column on the urgent communicator
(the reference's LOWER/UPPER tile shapes: half the bytes).
"""
from __future__ import annotations

import os

import torch

from ..constants import dplasmaConjTrans, dplasmaLeft, dplasmaLower, dplasmaNoTrans, dplasmaNonUnit, dplasmaRight
from ..ops import tile_ops as ops
from ..ops.batch import MASK_LOWER, MASK_UPPER, GemmBatch, TileBatch
from ..parallel import comm
from ..runtime import Taskpool
from ..utils.flops import flops

# distributed defaults (tools/replay_potrf.py decides them, profiles/r3_potrf_replay*.txt)
DIST_DEFER = 2
DIST_LOOKAHEAD = 2
DIST_BULK_RESERVE = 0
DIST_TILE_CUS = 0   # CUs kept for the diagonal-tile kernels (Context.partition_streams); 0 = no partition
DIST_CHUNK = 0      # D = 1: tiles per pipelined chunk (potrf_pipelined_New); 0 = whole-piece schedule (replay: chunking
#                   loses, 285 vs 241 ms at chunk 8 -- profiles/r3_replay_pipelined_chunks.txt)


class _Panel:
    def __init__(self, base, ld, off_fn):
        self.base, self.ld, self.off = base, ld, off_fn


def potrf_dist_New(ctx, uplo: int, A, info_out=None) -> Taskpool:
    lower = uplo == dplasmaLower
    tp = Taskpool("potrf", ctx)
    tp.flops = flops(A.prec, "potrf", A.n)
    nt = A.nt
    dev = A.device
    nbe = A.mb * A.nb
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    tp.info = info
    P, Q = A.P, A.Q
    env = os.environ
    D = max(1, int(env.get("DPLASMA_POTRF_DEFER", DIST_DEFER)))
    min_tiles = int(env.get("DPLASMA_POTRF_DEFER_MIN_TILES", 24))
    la = int(env.get("DPLASMA_POTRF_LOOKAHEAD", DIST_LOOKAHEAD))
    if la not in (1, 2):
        raise ValueError("DPLASMA_POTRF_LOOKAHEAD must be 1 or 2")
    nslab = 1 + la
    reserve = int(env.get("DPLASMA_POTRF_BULK_RESERVE", DIST_BULK_RESERVE))
    tile_cus = int(env.get("DPLASMA_POTRF_TILE_CUS", DIST_TILE_CUS))
    if tile_cus > 0 and ctx.is_gpu:
        # the diagonal tile (and a receiver's (M, S) preparation) on their own CUs, everything else on
        # the rest: the latency-bound tile kernels never share a SIMD with GEMM waves
        s_tile, s_chain, upd_stream = ctx.partition_streams(tile_cus)
        # a CU-masked stream has no priority: by default the chain keeps the high-priority panel stream
        s_pan = s_chain if env.get("DPLASMA_POTRF_CHAIN_MASKED", "0") == "1" else "panel"
    else:
        s_tile = s_pan = "panel"
        upd_stream = ctx.bulk_stream(reserve) if ctx.is_gpu else "update"
    chunk = int(env.get("DPLASMA_POTRF_CHUNK", DIST_CHUNK))
    if D == 1 and chunk > 0:
        return potrf_pipelined_New(ctx, uplo, A, info_out, chunk)
    if ctx.is_gpu and "comm" not in ctx.streams:
        ctx.streams["comm"] = torch.cuda.Stream(device=dev, priority=torch.cuda.Stream.priority_range()[1])
    urgent_g = ctx.urgent_group
    bulk_gs = ctx.bulk_groups or [None]

    # ---- axis abstraction: the panel of lower is a tile column spread over process rows ("lines");
    # upper is the transpose (a tile row spread over process columns)
    def line(i):
        return A.grid.prow(i + A.it0) if lower else A.grid.pcol(i + A.jt0)

    def cross(i):
        return A.grid.pcol(i + A.jt0) if lower else A.grid.prow(i + A.it0)

    def rank_lc(l, c):
        return A.grid.rank(l, c) if lower else A.grid.rank(c, l)

    def tcoord(i, k):
        return (i, k) if lower else (k, i)

    my_line = A.myrow if lower else A.mycol
    my_cross = A.mycol if lower else A.myrow
    nlines = P if lower else Q

    blocks = []
    c = 0
    while c < nt:
        d = D if nt - c >= min_tiles else 1
        blocks.append((c, min(nt, c + d)))
        c += d
    block_of = {}
    for b, (c0, c1) in enumerate(blocks):
        for k in range(c0, c1):
            block_of[k] = b

    # ---- per panel: every line's tiles sorted by (cross, i) (the packing order of its root)
    def line_tiles(k):
        per = [[] for _ in range(nlines)]
        for i in range(k + 1, nt):
            per[line(i)].append(i)
        for l in range(nlines):
            per[l].sort(key=lambda i: (cross(i), i))
        return per

    maxcnt = maxsub = 1
    for k in range(nt):
        per = line_tiles(k)
        maxcnt = max(maxcnt, max(len(p) for p in per))
        maxsub = max(maxsub, max(sum(1 for i in p if cross(i) == my_cross) for p in per))
    SG, SX = maxcnt * nbe, nlines * maxsub * nbe
    slab = SG + SX
    GX = torch.zeros(nslab * D * slab, dtype=A.dtype, device=dev)
    # loopback rehearsal (parallel.comm.loopback, world 1): the root packs its piece into LB and sends
    # it to itself into G, and the diagonal triangle goes to itself too -- the exchanges a real grid
    # has, through the same RCCL calls, with the receive-side paths (DRECV unpack, PREP) taken
    loop = bool(getattr(ctx, "loopback", False))
    me = ctx.rank
    LB = torch.zeros(nslab * D * SG if loop else 1, dtype=A.dtype, device=dev)
    ntri = A.mb * (A.mb + 1) // 2
    dsend = torch.zeros(2 * ntri, dtype=A.dtype, device=dev)
    drecv = torch.zeros(2 * ntri, dtype=A.dtype, device=dev)
    dbuf = torch.zeros(2 * nbe, dtype=A.dtype, device=dev)
    tp._buffers = (GX, dsend, drecv, dbuf, LB)

    use_rb = ops.rb_ok(A.data, A.mb) and A.mb == A.nb
    # panel TRSM: "rb" (register-resident strips, k_trsm_rb) or "gemm" (the batched TRSM engine: blocked
    # substitution on 16-blocks with MFMA updates, workgroups shaped like the bulk GEMM's)
    trsm_rb = use_rb and env.get("DPLASMA_POTRF_TRSM", "rb") == "rb"
    if use_rb:
        zsz = ops.rb_zbuf_size()
        zbufs = torch.empty(2 * zsz, dtype=torch.float64, device=dev)
        tp._zbufs = zbufs
    tri_mask = MASK_LOWER if lower else MASK_UPPER
    tA, tB = (dplasmaNoTrans, dplasmaConjTrans) if lower else (dplasmaConjTrans, dplasmaNoTrans)

    def window(k):
        """columns updated on the critical path by panel k: the rest of its block and the next one"""
        b = block_of[k]
        hi = blocks[b + 1][1] if b + 1 < len(blocks) else nt
        return range(k + 1, hi)

    def urgent_cross(k):
        return {cross(j) for j in window(k)}

    panels = {}
    # parity -> the last task of this rank that read the diagonal receive buffer of that parity: the next DRECV into it
    # waits for that reader (panel k-2 is another process column's when Q > 2, so "TRSM(k-2)" would not exist here --
    # found by tests/test_potrf_hazards.py)
    drecv_reader = {}
    pend = {}          # k -> {"u": Pending, "b": Pending} (this rank's batches of panel k)
    send_pend = {}     # slot -> list of Pending whose sends read that slab
    dsend_pend = {}    # k % 2 -> Pending of the diag send reading dsend[k % 2]

    def add_update(batch, ks, ncols):
        for n_ in ncols:
            for m_ in range(n_, nt):
                cc = (m_, n_) if lower else (n_, m_)
                if not A.is_local(*cc):
                    continue
                kp = [(panels[k].off(cc[0]), panels[k].off(cc[1]), A.tile_rows(k)) for k in ks]
                batch.add(A.offset(*cc), A.tile_rows(cc[0]), A.tile_cols(cc[1]), kp, tri_mask if m_ == n_ else 0)
        return batch.finalize()

    def f_upd(batch, base, ld):
        ops.gemm(tA, tB, -1.0, base, ld, base, ld, 1.0, A.data, A.ld, batch)

    # DPLASMA_POTRF_BULK_CAP=c: the bulk updates (NEXT2 / REST2) as capped grid-stride GEMM launches of
    # 2 x (CUs - c) workgroups (ops.gemm_wg_cap; the capped kernel no longer spills), so the panel chain's
    # kernels find free workgroup slots at once -- the single-process engine's DPLASMA_POTRF_RESERVE
    bulk_cap = 0
    cap_res = int(env.get("DPLASMA_POTRF_BULK_CAP", "0"))
    if cap_res > 0 and ctx.is_gpu:
        bulk_cap = 2 * max(8, torch.cuda.get_device_properties(dev).multi_processor_count - cap_res)

    def f_bulk(batch, base, ld):
        if bulk_cap:
            with ops.gemm_wg_cap(bulk_cap):
                f_upd(batch, base, ld)
        else:
            f_upd(batch, base, ld)

    def wait_panels(ks):
        # the consumer's stream waits for the receives of panels ks (never for this rank's sends)
        for k in ks:
            comm.finish(pend.get(k, {}).get("r"))

    gate = None
    last_upd = {}
    nxt2_of, rest_of = {}, {}
    last_panel = None
    slot_readers = {}   # slot -> tasks reading it (updates); the next user of the slot follows them
    for b, (c0, c1) in enumerate(blocks):
        par = b % nslab
        for k in range(c0, c1):
            kb = A.tile_rows(k)
            dk = tcoord(k, k)
            pc = cross(k)
            in_pc = my_cross == pc
            diag_line = line(k)
            own_diag = in_pc and my_line == diag_line
            per = line_tiles(k)
            mine = per[my_line] if in_pc else []
            slot = par * D + (k - c0)
            o = slot * slab
            guard = slot_readers.get(slot, [])
            # ---------------- POTRF(k)
            t_potrf = None
            zk = zbufs[(k % 2) * zsz:(k % 2 + 1) * zsz] if use_rb else None
            if own_diag:
                off = A.offset(*dk)

                def f_potrf(off=off, kb=kb, k=k, zk=zk):
                    if use_rb:
                        ops.potrf_tile(uplo, A.data, off, kb, A.ld, info, k * A.mb, zbuf=zk)
                    else:
                        ops.potrf_tile(uplo, A.data, off, kb, A.ld, info, k * A.mb)
                t_potrf = tp.task(f"POTRF({k})", s_tile, f_potrf, [gate], prio=3, comm=False)
            # ---------------- diagonal triangle to the other roots of the panel column
            tri_src = None
            t_dsend = None
            if in_pc and mine and not own_diag:
                src = rank_lc(diag_line, pc)
                par2 = k % 2

                def f_drecv(src=src, par2=par2, k=k, kb=kb):
                    h = comm.start_p2p(recvs=[(drecv[par2 * ntri:(par2 + 1) * ntri], src)], group=urgent_g,
                                       hint=("potrf", kb))
                    pend.setdefault(k, {})["d"] = h
                # the buffer pair alternates: panel k-2's TRSM must have read it (deps)
                t_dr = tp.task(f"DRECV({k})", "comm", f_drecv, [drecv_reader.get(par2)], prio=3)
                tri_src = (t_dr, par2)
            if own_diag:
                dests = [rank_lc(l, pc) for l in range(nlines) if l != my_line and per[l]]
                self_rx = loop and bool(mine)
                if dests or self_rx:
                    par2 = k % 2

                    def f_dsend(dests=dests, par2=par2, off=A.offset(*dk), kb=kb, k=k, self_rx=self_rx):
                        comm.finish(dsend_pend.get(par2))
                        buf = dsend[par2 * ntri:(par2 + 1) * ntri]
                        buf[: kb * (kb + 1) // 2].copy_(A.data.view(-1)[off + comm._tri_index(kb, A.ld, lower, dev)])
                        if self_rx:   # loopback: the triangle to myself, received like a remote root's
                            h = comm.start_p2p(sends=[(buf, me)], recvs=[(drecv[par2 * ntri:(par2 + 1) * ntri], me)],
                                               group=urgent_g)
                            pend.setdefault(k, {})["d"] = h
                        else:
                            h = comm.start_p2p(sends=[(buf, d) for d in dests], group=urgent_g)
                        dsend_pend[par2] = h
                    # (loopback: the receive buffer pair alternates as for DRECV)
                    t_dsend = tp.task(f"DSEND({k})", s_tile, f_dsend,
                                      [t_potrf] + ([drecv_reader.get(par2)] if self_rx else []), prio=3)
                    if self_rx:
                        tri_src = (t_dsend, par2)
            # ---------------- TRSM of my tiles of panel k
            t_trsm = None
            if mine:
                if tri_src is not None:
                    t_dr, par2 = tri_src
                    tri_base, tri_ld, tri_off = dbuf, A.mb, par2 * nbe

                    def f_unpack(par2=par2, kb=kb, k=k):
                        comm.finish(pend[k]["d"])
                        d = dbuf[par2 * nbe:(par2 + 1) * nbe]
                        d[comm._tri_index(kb, A.mb, lower, dev)] = drecv[par2 * ntri: par2 * ntri + kb * (kb + 1) // 2]
                    pre = [(f_unpack, t_dr)]
                else:
                    tri_base, tri_ld, tri_off = A.data, A.ld, A.offset(*dk)
                    pre = []
                if trsm_rb:
                    rbp = ops.RbPanel(uplo, [(A.offset(*tcoord(i, k)), A.tile_rows(i) if lower else A.tile_cols(i))
                                             for i in mine], A.ld)
                    prep = []
                    if pre:
                        # a receiver prepares (M, S) of the received triangle on the tile CUs
                        def f_prep(tb_=tri_base, tl=tri_ld, to=tri_off, kb=kb, zk=zk, pre=pre):
                            for f, _ in pre:
                                f()
                            ops.trsm_rb_prep(uplo, kb, tb_, to, tl, zk)
                        prep = [tp.task(f"PREP({k})", s_tile, f_prep, [gate] + [t for _, t in pre], prio=3,
                                        comm=False)]

                    def f_trsm(rbp=rbp, tb_=tri_base, tl=tri_ld, to=tri_off, kb=kb, zk=zk):
                        ops.trsm_rb(uplo, kb, tb_, to, tl, zk, rbp, A.data, A.ld)
                    deps = [t_potrf, gate] + prep
                else:
                    tb = TileBatch()
                    for i in mine:
                        cc = tcoord(i, k)
                        tb.add(tri_off, A.tile_rows(cc[0]), A.tile_cols(cc[1]), b_off=A.offset(*cc))
                    tb.finalize()
                    side = dplasmaRight if lower else dplasmaLeft

                    def f_trsm(tb=tb, tb_=tri_base, tl=tri_ld, side=side, pre=pre):
                        for f, _ in pre:
                            f()
                        ops.trsm(side, uplo, dplasmaConjTrans, dplasmaNonUnit, 1.0, tb_, tl, A.data, A.ld, tb)
                    deps = [t_potrf, gate] + [t for _, t in pre]
                t_trsm = tp.task(f"TRSM({k})", s_pan, f_trsm, deps, prio=2, comm=False)
                if tri_src is not None:
                    drecv_reader[tri_src[1]] = t_trsm
            if k == nt - 1:
                break
            # ---------------- panel k's transport
            ucross = urgent_cross(k)
            G = o
            X = o + SG
            # my receive layout: G = my line's piece (root's packing order); X[l] = line l's tiles of my cross
            pos_g = {i: j for j, i in enumerate(per[my_line])}
            pos_x = {}
            for l in range(nlines):
                if l == my_line:
                    continue
                sub = sorted(i for i in per[l] if cross(i) == my_cross)
                for j, i in enumerate(sub):
                    pos_x[i] = X + (l * maxsub + j) * nbe
            sends = {"u": [], "b": []}
            recvs = {"u": [], "b": []}
            me_urgent = my_cross in ucross
            if mine:
                # my piece -> G (packed by cross), then: my line's other crosses get all of it, every
                # other line's rank of cross c gets the sub-range of cross c
                for c_ in range(Q if lower else P):
                    if c_ == my_cross:
                        continue
                    kind = "u" if c_ in ucross else "b"
                    sends[kind].append((G, len(mine), rank_lc(my_line, c_)))
                for l in range(nlines):
                    if l == my_line:
                        continue
                    cs = {}
                    for j, i in enumerate(mine):
                        cs.setdefault(cross(i), []).append(j)
                    for c_, js in cs.items():
                        kind = "u" if c_ in ucross else "b"
                        sends[kind].append((G + js[0] * nbe, len(js), rank_lc(l, c_)))
            kind_me = "u" if me_urgent else "b"
            if loop and mine:
                # loopback: packed into LB, sent to myself into G (same batch: one group call)
                sends[kind_me].append((-1 - slot * SG, len(mine), me))
                recvs[kind_me].append((G, len(mine), me))
            if not in_pc and per[my_line]:
                recvs[kind_me].append((G, len(per[my_line]), rank_lc(my_line, pc)))
            for l in range(nlines):
                if l == my_line:
                    continue
                nsub = sum(1 for i in per[l] if cross(i) == my_cross)
                if nsub:
                    recvs[kind_me].append((X + l * maxsub * nbe, nsub, rank_lc(l, pc)))
            pack = None
            if mine:
                pb = TileBatch()
                pk0 = slot * SG if loop else G
                for j, i in enumerate(mine):
                    cc = tcoord(i, k)
                    pb.add(A.offset(*cc), A.tile_rows(cc[0]), A.tile_cols(cc[1]), b_off=pk0 + j * nbe)
                pack = pb.finalize()
            bg = bulk_gs[k % len(bulk_gs)]
            hint_row = ("trsm", len(per[my_line]), kb)

            def f_xfer(pack=pack, sends=sends, recvs=recvs, k=k, slot=slot, bg=bg, hint_row=hint_row):
                for h in send_pend.pop(slot, []):   # the slab's previous sends have read it
                    comm.finish(h)
                if pack is not None:
                    ops.geadd(0, dplasmaNoTrans, 1.0, A.data, A.ld, 0.0, LB if loop else GX, A.mb, pack, copy=True)
                hs = {}
                for kind, grp in (("u", urgent_g), ("b", bg)):
                    # a < 0: offset -1 - a in the loopback slab LB
                    s_ = [((LB[-1 - a: -1 - a + n * nbe] if a < 0 else GX[a: a + n * nbe]), r) for a, n, r in sends[kind]]
                    r_ = [(GX[a: a + n * nbe], r) for a, n, r in recvs[kind]]
                    if s_ or r_:
                        h = comm.start_p2p(s_, r_, group=grp, hint=hint_row)
                        if r_:
                            hs["r"] = h          # the batch carrying my receives (one kind per rank)
                        if s_:
                            send_pend.setdefault(slot, []).append(h)
                pend[k] = {**pend.get(k, {}), **hs}
            # a root issues after its TRSM (panel stream); a pure receiver on the comm stream, as soon
            # as the slab is free
            stream = s_pan if mine else "comm"
            t_x = tp.task(f"XFER({k})", stream, f_xfer, [t_trsm, *guard], prio=2)
            last_panel = t_x

            def poff(i, pos_g=pos_g, pos_x=pos_x, G=G):
                if line(i) == my_line:
                    return G + pos_g[i] * nbe
                return pos_x[i]
            panels[k] = _Panel(GX, A.mb, poff)
            base, ld = GX, A.mb
            # ---------------- NEAR(k): the rest of this block (panel stream)
            near = add_update(GemmBatch(), [k], range(k + 1, c1))
            if len(near):
                def f_near(bt=near, k=k):
                    wait_panels([k])
                    f_upd(bt, GX, A.mb)
                gate = tp.task(f"NEAR({k})", s_pan, f_near, [t_x, gate], prio=2, comm=False)
                slot_readers.setdefault(slot, []).append(gate)
            else:
                gate = t_x if t_x is not None else gate
        if c1 >= nt:
            break
        ks = list(range(c0, c1))
        n0, n1 = blocks[b + 1]
        my_slots = [par * D + (k - c0) for k in ks]
        if la == 1:
            nxt = add_update(GemmBatch(), ks, range(n0, n1))
            rest = add_update(GemmBatch(), ks, range(n1, nt))
            deps = [gate, last_panel, last_upd.get(b - 1)]
            t_next = None
            if len(nxt):
                def f_next(bt=nxt, ks=ks):
                    wait_panels(ks)
                    f_upd(bt, GX, A.mb)
                t_next = tp.task(f"NEXT({b})", upd_stream, f_next, deps, prio=2, comm=False)
                last_upd[b] = t_next
            if len(rest):
                def f_rest(bt=rest, ks=ks):
                    wait_panels(ks)
                    f_upd(bt, GX, A.mb)
                last_upd[b] = tp.task(f"REST({b})", upd_stream, f_rest, deps, prio=1, comm=False)
            for s_ in my_slots:
                slot_readers[s_] = [t for t in (last_upd.get(b), gate) if t is not None]
            gate = t_next if t_next is not None else gate
            continue
        n2 = blocks[b + 2][1] if b + 2 < len(blocks) else nt
        nxt = add_update(GemmBatch(), ks, range(n0, n1))
        nxt2 = add_update(GemmBatch(), ks, range(n1, n2))
        rest = add_update(GemmBatch(), ks, range(n2, nt))
        t_next = None
        if len(nxt):
            def f_next(bt=nxt, ks=ks):
                wait_panels(ks)
                f_upd(bt, GX, A.mb)
            t_next = tp.task(f"NEXT({b})", s_pan, f_next,
                             [gate, last_panel, nxt2_of.get(b - 1), rest_of.get(b - 2)], prio=2, comm=False)
        prev_bulk = rest_of.get(b - 1)
        if len(nxt2):
            def f_nxt2(bt=nxt2, ks=ks):
                wait_panels(ks)
                f_bulk(bt, GX, A.mb)
            nxt2_of[b] = tp.task(f"NEXT2({b})", upd_stream, f_nxt2, [gate, last_panel, prev_bulk], prio=1,
                                 comm=False)
        if len(rest):
            def f_rest(bt=rest, ks=ks):
                wait_panels(ks)
                f_bulk(bt, GX, A.mb)
            rest_of[b] = tp.task(f"REST2({b})", upd_stream, f_rest, [gate, last_panel, prev_bulk, nxt2_of.get(b)],
                                 prio=0, comm=False)
        else:
            rest_of[b] = nxt2_of.get(b, prev_bulk)
        last_upd[b] = rest_of[b] if rest_of[b] is not None else t_next
        for s_ in my_slots:
            slot_readers[s_] = [t for t in (last_upd.get(b), t_next, gate) if t is not None]
        gate = t_next if t_next is not None else gate

    def _done():
        # every exchange this rank started is complete before the buffers can be reused or freed
        for d in pend.values():
            for h in d.values():
                comm.finish(h)
        for hs in send_pend.values():
            for h in hs:
                comm.finish(h)
        for h in dsend_pend.values():
            comm.finish(h)
        pend.clear()
        send_pend.clear()
        dsend_pend.clear()
        v = info.clone()
        comm.allreduce(v, op=torch.distributed.ReduceOp.MAX)
        r = int(v.item())
        if r < 0:
            raise RuntimeError(f"potrf: tile kernel failure (info {r})")
        if info_out is not None:
            info_out[0] = r
        return r
    tp.on_complete(_done)
    return tp.finish_build()



def potrf_pipelined_New(ctx, uplo: int, A, info_out=None, chunk: int = 8) -> Taskpool:
    """Distributed Cholesky with the critical path pipelined at chunk granularity (one panel per
    step, look-ahead 2).  The replay (tools/replay_potrf.py, profiles/r3_replay_*) shows the
    whole-piece schedule above waiting, every panel, for the entire panel piece to reach the owners
    of the next column (up to 64 tiles = 128 MiB at N = 64k on 2 x 4): a transfer on the critical
    path.  Here each root solves, packs and sends its piece in chunks of ``chunk`` tiles (tile rows
    grouped by their position in the root's process row, so consecutive panels use the same row
    chunks), and the owners of column k+1 update it chunk by chunk as chunks arrive:

        TRSM(k, c) -> XFER_U(k, c) -> NEXT(k, c) -> TRSM(k+1, c) -> ...

    so the next diagonal tile (always in the first chunk) is ready after one chunk's latency, and
    the rest of the piece streams behind it -- the tile-granular pipelining PaRSEC gets from its
    per-tile remote dependencies (zpotrf_L.jdf:209-217).  Ranks that do not own column k+1 get the
    piece as one bulk message on a bulk communicator; NEXT2 (column k+2) and REST2 (beyond) run on
    the bulk stream after the whole panel has arrived."""
    lower = uplo == dplasmaLower
    tp = Taskpool("potrf", ctx)
    tp.flops = flops(A.prec, "potrf", A.n)
    nt = A.nt
    dev = A.device
    nbe = A.mb * A.nb
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    tp.info = info
    P, Q = A.P, A.Q
    C = max(1, int(chunk))
    NSLAB = 3
    reserve = int(os.environ.get("DPLASMA_POTRF_BULK_RESERVE", DIST_BULK_RESERVE))
    upd_stream = ctx.bulk_stream(reserve) if ctx.is_gpu else "update"
    if ctx.is_gpu and "comm" not in ctx.streams:
        ctx.streams["comm"] = torch.cuda.Stream(device=dev, priority=torch.cuda.Stream.priority_range()[1])
    urgent_g = ctx.urgent_group
    bulk_gs = ctx.bulk_groups or [None]

    def line(i):
        return A.grid.prow(i + A.it0) if lower else A.grid.pcol(i + A.jt0)

    def cross(i):
        return A.grid.pcol(i + A.jt0) if lower else A.grid.prow(i + A.it0)

    def rank_lc(l, c_):
        return A.grid.rank(l, c_) if lower else A.grid.rank(c_, l)

    def tcoord(i, k):
        return (i, k) if lower else (k, i)

    my_line = A.myrow if lower else A.mycol
    my_cross = A.mycol if lower else A.myrow
    nlines = P if lower else Q
    ncross = Q if lower else P
    # chunk of a tile row: its position among its line's tile rows, in groups of C
    pos_line, cnt_line = {}, [0] * nlines
    for i in range(nt):
        pos_line[i] = cnt_line[line(i)]
        cnt_line[line(i)] += 1

    def chunk_of(i):
        return pos_line[i] // C

    def piece(k, l):
        return [i for i in range(k + 1, nt) if line(i) == l]

    maxcnt = max(1, max(len(piece(0, l)) for l in range(nlines)))
    maxsub = max(1, max(sum(1 for i in piece(0, l) if cross(i) == my_cross) for l in range(nlines)))
    # slab: G (my line's piece by row), XS (my piece regrouped by destination cross, root only),
    # XR[l] (line l's tiles of my cross, by row)
    SG, SXS, SXR = maxcnt * nbe, maxcnt * nbe, nlines * maxsub * nbe
    slab = SG + SXS + SXR
    GX = torch.zeros(NSLAB * slab, dtype=A.dtype, device=dev)
    ntri = A.mb * (A.mb + 1) // 2
    dsend = torch.zeros(2 * ntri, dtype=A.dtype, device=dev)
    drecv = torch.zeros(2 * ntri, dtype=A.dtype, device=dev)
    dbuf = torch.zeros(2 * nbe, dtype=A.dtype, device=dev)
    tp._buffers = (GX, dsend, drecv, dbuf)
    use_rb = ops.rb_ok(A.data, A.mb) and A.mb == A.nb
    # panel TRSM: "rb" (register-resident strips, k_trsm_rb) or "gemm" (the batched TRSM engine: blocked
    # substitution on 16-blocks with MFMA updates, workgroups shaped like the bulk GEMM's)
    trsm_rb = use_rb and os.environ.get("DPLASMA_POTRF_TRSM", "rb") == "rb"
    if use_rb:
        zsz = ops.rb_zbuf_size()
        zbufs = torch.empty(2 * zsz, dtype=torch.float64, device=dev)
        tp._zbufs = zbufs
    tri_mask = MASK_LOWER if lower else MASK_UPPER
    tA, tB = (dplasmaNoTrans, dplasmaConjTrans) if lower else (dplasmaConjTrans, dplasmaNoTrans)

    pend = {}          # (k, tag) -> Pending carrying my receives ("d", ("u", c), "b")
    send_pend = {}     # slot -> Pendings whose sends read the slab
    dsend_pend = {}
    poffs = {}         # k -> offset function of panel k's tiles

    def f_upd(batch):
        ops.gemm(tA, tB, -1.0, GX, A.mb, GX, A.mb, 1.0, A.data, A.ld, batch)

    def upd_batch(k, ncols, rows=None):
        """C(m, n) -= L(m, k) L(n, k)^H for my tiles, n in ncols, m >= n (m in rows if given)."""
        b = GemmBatch()
        off = poffs[k]
        for n_ in ncols:
            for m_ in range(n_, nt):
                if rows is not None and m_ not in rows:
                    continue
                cc = (m_, n_) if lower else (n_, m_)
                if not A.is_local(*cc):
                    continue
                b.add(A.offset(*cc), A.tile_rows(cc[0]), A.tile_cols(cc[1]), [(off(cc[0]), off(cc[1]), A.tile_rows(k))],
                      tri_mask if m_ == n_ else 0)
        return b.finalize()

    nxt_chunk = {}     # (k, chunk) -> NEXT(k, chunk) task on this rank
    nxt2 = {}          # k -> NEXT2(k)
    rest2 = {}         # k -> REST2(k)
    drecv_reader = {}   # parity -> the last reader of that diagonal receive buffer on this rank (see potrf_dist_New)
    slot_readers = {}
    for k in range(nt):
        kb = A.tile_rows(k)
        dk = tcoord(k, k)
        pc = cross(k)
        in_pc = my_cross == pc
        diag_line = line(k)
        own_diag = in_pc and my_line == diag_line
        mine = piece(k, my_line) if in_pc else []
        slot = k % NSLAB
        o = slot * slab
        G, XS, XR = o, o + SG, o + SG + SXS
        guard = slot_readers.get(slot, [])
        col_deps = [nxt2.get(k - 2)]          # column k's last bulk update (NEXT2(k-2), after REST2(k-3))
        zk = zbufs[(k % 2) * zsz:(k % 2 + 1) * zsz] if use_rb else None
        # ---------------- POTRF(k)
        t_potrf = None
        if own_diag:
            off = A.offset(*dk)

            def f_potrf(off=off, kb=kb, k=k, zk=zk):
                if use_rb:
                    ops.potrf_tile(uplo, A.data, off, kb, A.ld, info, k * A.mb, zbuf=zk)
                else:
                    ops.potrf_tile(uplo, A.data, off, kb, A.ld, info, k * A.mb)
            t_potrf = tp.task(f"POTRF({k})", "panel", f_potrf, [nxt_chunk.get((k - 1, chunk_of(k))), *col_deps],
                              prio=3, comm=False)
        # ---------------- diagonal triangle to the other roots of column pc
        t_dr = None
        if in_pc and mine and not own_diag:
            src = rank_lc(diag_line, pc)
            par2 = k % 2

            def f_drecv(src=src, par2=par2, k=k, kb=kb):
                pend[(k, "d")] = comm.start_p2p(recvs=[(drecv[par2 * ntri:(par2 + 1) * ntri], src)], group=urgent_g,
                                                hint=("potrf", kb))
            t_dr = tp.task(f"DRECV({k})", "comm", f_drecv, [drecv_reader.get(par2)], prio=3)
        if own_diag:
            dests = [rank_lc(l, pc) for l in range(nlines) if l != my_line and piece(k, l)]
            if dests:
                par2 = k % 2

                def f_dsend(dests=dests, par2=par2, off=A.offset(*dk), kb=kb):
                    comm.finish(dsend_pend.get(par2))
                    buf = dsend[par2 * ntri:(par2 + 1) * ntri]
                    buf[: kb * (kb + 1) // 2].copy_(A.data.view(-1)[off + comm._tri_index(kb, A.ld, lower, dev)])
                    dsend_pend[par2] = comm.start_p2p(sends=[(buf, d) for d in dests], group=urgent_g)
                tp.task(f"DSEND({k})", "panel", f_dsend, [t_potrf], prio=3)
        if k == nt - 1:
            break
        # ---------------- layout of panel k on this rank
        j1 = k + 1
        ucross = cross(j1)                    # the owners of column k+1 are urgent
        urgent_me = my_cross == ucross
        pos_g = {i: t for t, i in enumerate(piece(k, my_line))}
        xr_pos, xr_rows = {}, {}
        for l in range(nlines):
            if l == my_line:
                continue
            sub = [i for i in piece(k, l) if cross(i) == my_cross]
            xr_rows[l] = sub
            for t, i in enumerate(sub):
                xr_pos[i] = XR + (l * maxsub + t) * nbe

        def poff(i, pos_g=pos_g, xr_pos=xr_pos, G=G):
            if line(i) == my_line:
                return G + pos_g[i] * nbe
            return xr_pos[i]
        poffs[k] = poff
        # root: XS = my piece regrouped by destination cross (each cross contiguous, rows ascending)
        xs_pos, xs_start = {}, {}
        if mine:
            p_ = 0
            for c_ in range(ncross):
                xs_start[c_] = p_
                for i in mine:
                    if cross(i) == c_:
                        xs_pos[i] = p_
                        p_ += 1
        chunks = sorted({chunk_of(i) for l in range(nlines) for i in piece(k, l)})
        # ---------------- per chunk: TRSM + pack (roots), urgent exchange, NEXT (column k+1 owners)
        trsm_tasks = []
        trsm_of = {}       # chunk -> TRSM(k, chunk) on this rank
        u_tasks = {}
        first = True
        t_first = None
        for c in chunks:
            ch = [i for i in mine if chunk_of(i) == c]
            t_tc = None
            if ch:
                pre = []
                if t_dr is not None and first:
                    par2 = k % 2

                    def f_unpack(par2=par2, kb=kb, k=k, zk=zk):
                        comm.finish(pend[(k, "d")])
                        d = dbuf[par2 * nbe:(par2 + 1) * nbe]
                        d[comm._tri_index(kb, A.mb, lower, dev)] = drecv[par2 * ntri: par2 * ntri + kb * (kb + 1) // 2]
                        if trsm_rb:
                            ops.trsm_rb_prep(uplo, kb, dbuf, par2 * nbe, A.mb, zk)
                    pre.append(f_unpack)
                if t_dr is not None:
                    tri_base, tri_ld, tri_off = dbuf, A.mb, (k % 2) * nbe
                else:
                    tri_base, tri_ld, tri_off = A.data, A.ld, A.offset(*dk)
                pk = TileBatch()
                for i in ch:
                    cc = tcoord(i, k)
                    pk.add(A.offset(*cc), A.tile_rows(cc[0]), A.tile_cols(cc[1]), b_off=G + pos_g[i] * nbe)
                    pk.add(A.offset(*cc), A.tile_rows(cc[0]), A.tile_cols(cc[1]), b_off=XS + xs_pos[i] * nbe)
                pk.finalize()
                if trsm_rb:
                    rbp = ops.RbPanel(uplo, [(A.offset(*tcoord(i, k)), A.tile_rows(i) if lower else A.tile_cols(i))
                                             for i in ch], A.ld)

                    def f_tc(rbp=rbp, tb_=tri_base, tl=tri_ld, to=tri_off, kb=kb, zk=zk, pre=pre, pk=pk, slot=slot,
                             firstc=first):
                        for f in pre:
                            f()
                        if firstc:
                            for h in send_pend.pop(slot, []):   # the slab's previous sends have read it
                                comm.finish(h)
                        ops.trsm_rb(uplo, kb, tb_, to, tl, zk, rbp, A.data, A.ld)
                        ops.geadd(0, dplasmaNoTrans, 1.0, A.data, A.ld, 0.0, GX, A.mb, pk, copy=True)
                else:
                    tb = TileBatch()
                    for i in ch:
                        cc = tcoord(i, k)
                        tb.add(tri_off, A.tile_rows(cc[0]), A.tile_cols(cc[1]), b_off=A.offset(*cc))
                    tb.finalize()
                    side = dplasmaRight if lower else dplasmaLeft

                    def f_tc(tb=tb, tb_=tri_base, tl=tri_ld, side=side, pre=pre, pk=pk, slot=slot, firstc=first):
                        for f in pre:
                            f()
                        if firstc:
                            for h in send_pend.pop(slot, []):
                                comm.finish(h)
                        ops.trsm(side, uplo, dplasmaConjTrans, dplasmaNonUnit, 1.0, tb_, tl, A.data, A.ld, tb)
                        ops.geadd(0, dplasmaNoTrans, 1.0, A.data, A.ld, 0.0, GX, A.mb, pk, copy=True)
                # later chunks follow the first (it unpacks the received triangle)
                deps = [t_potrf, t_dr, t_first, nxt_chunk.get((k - 1, c)), *col_deps, *guard]
                t_tc = tp.task(f"TRSM({k},{c})", "panel", f_tc, deps, prio=2, comm=False)
                trsm_tasks.append(t_tc)
                trsm_of[c] = t_tc
                if t_dr is not None:
                    drecv_reader[k % 2] = t_tc
                if first:
                    t_first = t_tc
                first = False
            # urgent exchange of chunk c: root sends to the column-(k+1) owners; they receive
            sends, recvs = [], []
            if ch:
                a, b_ = pos_g[ch[0]], pos_g[ch[-1]] + 1
                for c_ in range(ncross):
                    if c_ == my_cross or c_ != ucross:
                        continue
                    sends.append((GX[G + a * nbe: G + b_ * nbe], rank_lc(my_line, c_)))
                for l in range(nlines):
                    if l == my_line:
                        continue
                    sub = [xs_pos[i] for i in ch if cross(i) == ucross]
                    if sub:
                        sends.append((GX[XS + sub[0] * nbe: XS + (sub[-1] + 1) * nbe], rank_lc(l, ucross)))
            if urgent_me:
                if not in_pc:
                    gch = [i for i in piece(k, my_line) if chunk_of(i) == c]
                    if gch:
                        a, b_ = pos_g[gch[0]], pos_g[gch[-1]] + 1
                        recvs.append((GX[G + a * nbe: G + b_ * nbe], rank_lc(my_line, pc)))
                for l, sub in xr_rows.items():
                    sc = [t for t, i in enumerate(sub) if chunk_of(i) == c]
                    if sc:
                        base_ = XR + l * maxsub * nbe
                        recvs.append((GX[base_ + sc[0] * nbe: base_ + (sc[-1] + 1) * nbe], rank_lc(l, pc)))
            if sends or recvs:
                def f_xu(sends=sends, recvs=recvs, k=k, c=c, slot=slot, j1=j1):
                    h = comm.start_p2p(sends, recvs, group=urgent_g, hint=("trsm", C, A.tile_rows(j1)))
                    if recvs:
                        pend[(k, ("u", c))] = h
                    if sends:
                        send_pend.setdefault(slot, []).append(h)
                u_tasks[c] = tp.task(f"XFER_U({k},{c})", "panel" if ch else "comm", f_xu,
                                     [t_tc] if ch else list(guard), prio=2)
        # ---------------- bulk exchange of panel k: every non-urgent destination, whole
        sends, recvs = [], []
        if mine:
            for c_ in range(ncross):
                if c_ == my_cross or c_ == ucross:
                    continue
                sends.append((GX[G: G + len(mine) * nbe], rank_lc(my_line, c_)))
            for l in range(nlines):
                if l == my_line:
                    continue
                for c_ in range(ncross):
                    if c_ == ucross:
                        continue
                    n_ = sum(1 for i in mine if cross(i) == c_)
                    if n_:
                        s0 = xs_start[c_]
                        sends.append((GX[XS + s0 * nbe: XS + (s0 + n_) * nbe], rank_lc(l, c_)))
        if not urgent_me:
            if not in_pc and piece(k, my_line):
                recvs.append((GX[G: G + len(piece(k, my_line)) * nbe], rank_lc(my_line, pc)))
            for l, sub in xr_rows.items():
                if sub:
                    base_ = XR + l * maxsub * nbe
                    recvs.append((GX[base_: base_ + len(sub) * nbe], rank_lc(l, pc)))
        bg = bulk_gs[k % len(bulk_gs)]
        t_xb = None
        if sends or recvs:
            def f_xb(sends=sends, recvs=recvs, k=k, slot=slot, bg=bg, cnt=len(piece(k, my_line)), kb=kb):
                h = comm.start_p2p(sends, recvs, group=bg, hint=("trsm", cnt, kb))
                if recvs:
                    pend[(k, "b")] = h
                if sends:
                    send_pend.setdefault(slot, []).append(h)
            t_xb = tp.task(f"XFER_B({k})", "panel" if mine else "comm", f_xb,
                           (trsm_tasks[-1:] if mine else list(guard)) + list(u_tasks.values())[-1:], prio=1)

        def wait_all(k=k):
            for key in list(pend):
                if key[0] == k and key[1] != "d":
                    comm.finish(pend[key])
        # ---------------- NEXT(k, c): column k+1 on its owners, chunk by chunk
        readers = []
        if urgent_me:
            c0 = chunk_of(j1)      # the chunk carrying L(k+1, k), the column operand of every row
            for c in chunks:
                rows = {i for i in piece(k, my_line) if chunk_of(i) == c}
                bt = upd_batch(k, [j1], rows)
                if not len(bt):
                    continue

                def f_next(bt=bt, k=k, c=c, c0=c0):
                    comm.finish(pend.get((k, ("u", c))))
                    comm.finish(pend.get((k, ("u", c0))))
                    f_upd(bt)
                # (a root -- Q = 1 grids -- reads its own packed chunks c and c0)
                deps = [u_tasks.get(c), u_tasks.get(c0), trsm_of.get(c), trsm_of.get(c0), nxt2.get(k - 1)]
                t = tp.task(f"NEXT({k},{c})", "panel", f_next, deps, prio=2, comm=False)
                nxt_chunk[(k, c)] = t
                readers.append(t)
        # ---------------- NEXT2(k) (column k+2) and REST2(k) (beyond) on the bulk stream
        last_x = t_xb if t_xb is not None else (list(u_tasks.values())[-1] if u_tasks else None)
        prev_bulk = rest2.get(k - 1)
        if k + 2 < nt:
            bt2 = upd_batch(k, [k + 2])
            if len(bt2):
                def f_n2(bt=bt2, wait_all=wait_all):
                    wait_all()
                    f_upd(bt)
                nxt2[k] = tp.task(f"NEXT2({k})", upd_stream, f_n2, [last_x, prev_bulk], prio=1, comm=False)
        if k + 3 < nt:
            br = upd_batch(k, range(k + 3, nt))
            if len(br):
                def f_r2(bt=br, wait_all=wait_all):
                    wait_all()
                    f_upd(bt)
                rest2[k] = tp.task(f"REST2({k})", upd_stream, f_r2, [last_x, prev_bulk, nxt2.get(k)], prio=0,
                                   comm=False)
        if k not in rest2:
            rest2[k] = nxt2.get(k, prev_bulk)
        if k not in nxt2:
            nxt2[k] = prev_bulk
        slot_readers[slot] = [t for t in readers + [rest2.get(k), nxt2.get(k), last_x] if t is not None]

    def _done():
        for h in list(pend.values()):
            comm.finish(h)
        for hs in send_pend.values():
            for h in hs:
                comm.finish(h)
        for h in dsend_pend.values():
            comm.finish(h)
        pend.clear()
        send_pend.clear()
        dsend_pend.clear()
        v = info.clone()
        comm.allreduce(v, op=torch.distributed.ReduceOp.MAX)
        r = int(v.item())
        if r < 0:
            raise RuntimeError(f"potrf: tile kernel failure (info {r})")
        if info_out is not None:
            info_out[0] = r
        return r
    tp.on_complete(_done)
    return tp.finish_build()
