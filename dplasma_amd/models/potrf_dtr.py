"""Cholesky as ONE persistent launch of the device task runtime (``csrc/kernels/dtr.hip``).

The reference's Cholesky is a PTG whose POTRF / TRSM / HERK / GEMM task classes are scheduled by
PaRSEC with priorities: the panel classes are ``high_priority`` (``src/zpotrf_L.jdf:58-69, 93, 194,
306``), so a freed core or GPU stream takes panel work before trailing updates.  Stream priorities
cannot do that on MI355X: the bulk update GEMM holds every CU's VGPRs and LDS, and a panel kernel on a
high-priority stream is not even dispatched until the GEMM drains (``profiles/r4_prio_probe.txt``).
This builder compiles the factorisation into a device task table instead:

* tasks (one 256-thread workgroup each): ``POTRF(k, b)`` (row block b of the dataflow tile Cholesky
  of tile (k, k), then block column b of ``W_k = L_kk^{-T}``; 16 cooperating workgroups),
  ``TRSM(i, k, r)`` (128-row strip r of L(i, k) = A(i, k) W_k, a GEMM solved in place) and
  ``UPD(i, j, r, c, k0, nk)`` (128x128 sub-tile of the trailing update by a run of ``nk`` panels);
* panels are grouped in blocks of ``D`` (the deferred update of ``models/potrf.py``): inside a block
  each panel updates the block's remaining columns (``NEAR``), and the block then updates every later
  column with one k-run of ``D`` panels (``BULK``);
* dependencies are version counters of 128x128 sub-tiles (this builder simulates the sequential
  program once to know which version each task needs);
* the high-priority list (ordered by target column, then: the diagonal tile's updates, POTRF, the
  column's other updates, its TRSM strips) holds every panel task and the updates of the next block's
  columns; the low-priority lists (one per XCD, tiles of column j on XCD j mod 8, ordered by block
  then column) hold the rest of the bulk update.  Every workgroup takes the next ready high-priority
  task before any low-priority one.

One process, lower, fp64, NB = 512, N a multiple of 512 (``supported``); ``models/potrf.py`` uses it
when ``DPLASMA_POTRF_ENGINE=dtr`` (or ``auto`` and supported).
"""
from __future__ import annotations

import os
import struct
from typing import List

import numpy as np
import torch

from ..constants import dplasmaLower
from ..runtime.taskpool import Taskpool
from ..utils.flops import flops

NBT = 512
MAXB = 16
BLK = 32 * 32
RB = 32

TASK_DT = np.dtype([("type", "<i4"), ("i", "<i4"), ("j", "<i4"), ("k0", "<i4"), ("req_beg", "<i4"),
                    ("inc", "<i4"), ("r", "<i2"), ("c", "<i2"), ("nk", "<i2"), ("nreq", "<i2")])
assert TASK_DT.itemsize == 32
T_UPD, T_TRSM, T_POTRF = 0, 1, 2


def supported(ctx, uplo, A) -> bool:
    if not (ctx.is_gpu and ctx.world == 1 and not getattr(ctx, "loopback", False)):
        return False
    if uplo != dplasmaLower or A.dtype != torch.float64 or A.mb != NBT or A.nb != NBT:
        return False
    if A.m != A.n or A.m % NBT or A.m == 0 or A.data.device.type != "cuda":
        return False
    if getattr(A, "it0", 0) or getattr(A, "jt0", 0):
        return False
    si, sj = _strides(A)
    return si is not None


def _strides(A):
    """(si, sj) with A.offset(i, j) == i * si + j * sj for every tile, or (None, None)."""
    nt = A.nt
    si = A.offset(1, 0) - A.offset(0, 0) if nt > 1 else NBT
    sj = A.offset(0, 1) - A.offset(0, 0) if nt > 1 else NBT * A.ld
    if A.offset(0, 0) != 0:
        return None, None
    for (i, j) in ((nt - 1, 0), (0, nt - 1), (nt - 1, nt - 1), (nt // 2, nt // 3)):
        if A.offset(i, j) != i * si + j * sj:
            return None, None
    return si, sj


def _head_env(default: str = "") -> tuple:
    """DPLASMA_DTR_HEAD: comma-separated widths of the first panel blocks (then DPLASMA_DTR_DEFER)."""
    s = os.environ.get("DPLASMA_DTR_HEAD", default).strip()
    return tuple(int(x) for x in s.split(",") if x.strip())


class _Plan:
    """The task table of one factorisation (identical for every run of the same shape)."""

    def __init__(self, nt: int, D: int, lo_order: str = None, min_tiles: int = None, head=None):
        # low-list order: "panel" -- (last panel block, column, ...): the bulk runs breadth-first, block by
        # block; "column" -- (column block, last panel block, column, ...): a column block's remaining old
        # updates before the next column block's, so the first panel of a block does not wait behind the
        # whole previous bulk.  Both are subsequences of one topological order (column blocks ascending; in
        # a block, its low-list updates, then its high-list tasks), which the deadlock argument needs.
        # "deadline": BOTH lists ordered by the step at which a task's output is first needed on the critical
        # chain -- tile row i: an update of (i, j), i > j, and TRSM(i, k) feed TRSM(i, i-1) at step i - 1, the
        # diagonal tile's updates feed POTRF(i) at step i -- then column, phase (diagonal updates, POTRF,
        # other updates, TRSM), last panel.  One key for both lists, and a topological order: each task's
        # inputs have a smaller deadline, or the same deadline and a smaller column or phase.  The column-
        # major high list hands the tickets of a whole column's updates out before that column's first TRSM,
        # which puts every row of a column on the critical chain (profiles/r5_dtr_dist_emulation.txt).
        # "rowpipe": the column order, but inside a column the high list runs row by row -- the updates of
        # tile (i, j), then its TRSM strips (and their sends) -- so TRSM(j+1, j) waits for row j+1's inputs
        # only, not for the whole column's (a distributed grid receives the previous panel's strips row by
        # row; the in-order tickets would otherwise put the entire previous panel on the critical chain)
        # "step": both lists by the panel step that makes a task ready -- POTRF(k), W_k's sends, the TRSMs of
        # panel k (row by row, each strip followed by its sends), then every update whose run ends at panel k
        # (column by column: the next diagonal tile first).  An update is placed where its inputs appear, not
        # under its output column (the column order parks the look-ahead update of the next block's first
        # diagonal tile behind that block's panels: profiles/r5_dtr_dist_emulation.txt).
        lo_order = lo_order or os.environ.get("DPLASMA_DTR_LO_ORDER", "column")
        if lo_order not in ("panel", "column", "deadline", "rowpipe", "step"):
            raise ValueError("DPLASMA_DTR_LO_ORDER must be panel, column, rowpipe, step or deadline")
        self.order = lo_order
        dl = lo_order == "deadline"
        rp = lo_order == "rowpipe"
        sp = lo_order == "step"
        S = 4 * nt
        self.nt, self.S, self.D = nt, S, D
        # blocks of D panels; single panels once fewer than min_tiles columns remain (the chain-bound tail:
        # the stream engine's POTRF_DEFER_MIN_TILES rule)
        if min_tiles is None:
            min_tiles = int(os.environ.get("DPLASMA_DTR_DEFER_MIN_TILES", "0"))
        # head: the widths of the first blocks (then D).  A block's bulk update of the later columns waits for its
        # last panel, so with D = 4 from the start the first ~4 panels run with only their look-ahead work beside
        # them (dtr_trace_run.py 16k: ~1/3 of the workgroups busy over the first 15 % of the span)
        if head is None:
            head = _head_env()
        head = [max(1, int(h)) for h in head]
        blocks = []
        b0 = 0
        while b0 < nt:
            d = D if nt - b0 >= min_tiles else 1
            if len(blocks) < len(head):
                d = head[len(blocks)]
            blocks.append((b0, min(nt, b0 + d)))
            b0 += d
        block_of = np.zeros(nt, dtype=np.int64)
        for bi, (x0, x1) in enumerate(blocks):
            block_of[x0:x1] = bi
        self.blocks = blocks
        WB = S * S                      # counter index of W_k's "block columns done" count
        self.ncnt = WB + nt
        ver = np.zeros(S * S, dtype=np.int32)
        F = np.zeros((S, nt), dtype=np.int32)   # strip (I, k) solved: the value of its marker counter
        chunks, hi_parts, lo_parts = [], [], []
        key_parts = []      # (ids, key padded to 6 columns): the list order key of every task
        ntask = [0]

        def sc(I, J):
            return np.asarray(I, dtype=np.int64) + np.asarray(J, dtype=np.int64) * S

        def emit(typ, i, j, k0, r, c, nk, inc, reqs, nreq, prio, key=None, xcd=None):
            n = len(i)
            t = np.zeros(n, dtype=TASK_DT)
            t["type"], t["i"], t["j"], t["k0"] = typ, i, j, k0
            t["r"], t["c"], t["nk"], t["inc"] = r, c, nk, inc
            ids = np.arange(ntask[0], ntask[0] + n, dtype=np.int64)
            ntask[0] += n
            chunks.append((t, reqs, nreq))
            kk = np.zeros((n, 6), dtype=np.int64)
            kk[:, :key.shape[1]] = key
            key_parts.append(kk)
            if prio == "hi":
                hi_parts.append((key, ids))
            else:
                lo_parts.append((xcd, key, ids))
            return ids

        # sub-tile enumeration of tiles (i, j), i >= j: every (r, c), diagonal tiles only r >= c
        rr, cc = np.meshgrid(np.arange(4), np.arange(4), indexing="ij")
        rr, cc = rr.ravel(), cc.ravel()
        low = rr >= cc

        def subtiles(i, j):
            """i, j: tile index arrays -> (i, j, r, c) per sub-tile."""
            i, j = np.asarray(i), np.asarray(j)
            n = len(i)
            I = np.repeat(i, 16)
            J = np.repeat(j, 16)
            R = np.tile(rr, n)
            C = np.tile(cc, n)
            keep = (I != J) | np.tile(low, n)
            return I[keep], J[keep], R[keep], C[keep]

        def upd(i, j, r, c, k0, nk, prio_hi):
            """update tasks (arrays) by panels [k0, k0+nk); bumps the sub-tile versions."""
            n = len(i)
            width = 1 + 2 * nk
            reqs = np.full((n, width, 2), -1, dtype=np.int64)
            Ci = sc(4 * i + r, 4 * j + c)
            reqs[:, 0, 0], reqs[:, 0, 1] = Ci, ver[Ci]
            diag = (i == j) & (r == c)
            for q in range(nk):
                k = k0 + q
                a = sc(4 * i + r, 4 * k)
                b = sc(4 * j + c, 4 * k)
                reqs[:, 1 + 2 * q, 0], reqs[:, 1 + 2 * q, 1] = a, F[4 * i + r, k]
                reqs[:, 2 + 2 * q, 0] = np.where(diag, -1, b)
                reqs[:, 2 + 2 * q, 1] = np.where(diag, -1, F[4 * j + c, k])
            ver[Ci] += 1
            kl = k0 + nk - 1
            if sp:
                key = np.stack([np.full(n, kl), np.full(n, 3), j, i, r, c], 1)
                if prio_hi:
                    return emit(T_UPD, i, j, k0, r, c, nk, Ci, reqs, None, "hi", key=key)
                return emit(T_UPD, i, j, k0, r, c, nk, Ci, reqs, None, "lo", key=key, xcd=j % 8)
            if dl:
                key = np.stack([np.where(i == j, i, i - 1), j, np.where(i == j, 0, 2), np.full(n, kl), r, c], 1)
                if prio_hi:
                    return emit(T_UPD, i, j, k0, r, c, nk, Ci, reqs, None, "hi", key=key)
                return emit(T_UPD, i, j, k0, r, c, nk, Ci, reqs, None, "lo", key=key, xcd=j % 8)
            if prio_hi and rp:
                # key: column, phase (0 diagonal tile, 2 other rows), row, 0 (before the row's TRSM), last panel,
                # sub-tile
                key = np.stack([j, np.where(i == j, 0, 2), np.where(i == j, 0, i), np.zeros(n, int),
                                np.full(n, kl), 4 * r + c], 1)
                return emit(T_UPD, i, j, k0, r, c, nk, Ci, reqs, None, "hi", key=key)
            if prio_hi:
                # key: column, phase (0 diagonal tile, 2 other rows), last panel, row, sub-tile
                key = np.stack([j, np.where(i == j, 0, 2), np.full(n, kl), i, r, c], 1)
                return emit(T_UPD, i, j, k0, r, c, nk, Ci, reqs, None, "hi", key=key)
            if lo_order in ("column", "rowpipe"):
                key = np.stack([block_of[j], np.full(n, kl), j, i, r, c], 1)
            else:
                key = np.stack([np.full(n, kl), j, i, r, c], 1)
            return emit(T_UPD, i, j, k0, r, c, nk, Ci, reqs, None, "lo", key=key, xcd=j % 8)

        for bi, (k0b, k1b) in enumerate(blocks):
            for k in range(k0b, k1b):
                # POTRF(k, b): the diagonal tile's final versions (every update of it precedes)
                dI, dJ = np.meshgrid(np.arange(4), np.arange(4), indexing="ij")
                sel = dI >= dJ
                dsc = sc(4 * k + dI[sel], 4 * k + dJ[sel])
                reqs = np.full((MAXB, len(dsc), 2), -1, dtype=np.int64)
                reqs[:, :, 0] = dsc
                reqs[:, :, 1] = ver[dsc]
                b = np.arange(MAXB)
                if sp:
                    key = np.stack([np.full(MAXB, k), b * 0, b * 0, b * 0, b, b * 0], 1)
                elif dl:
                    key = np.stack([np.full(MAXB, k), np.full(MAXB, k), np.ones(MAXB, int), b * 0, b, b * 0], 1)
                else:
                    key = np.stack([np.full(MAXB, k), np.ones(MAXB, int), np.zeros(MAXB, int), b, b * 0, b * 0], 1)
                emit(T_POTRF, np.full(MAXB, k), np.full(MAXB, k), k, b, 0, 0, WB + k, reqs, None, "hi", key=key)
                if k + 1 < nt:
                    # TRSM(i, k, r): W_k complete and every update of strip r of tile (i, k)
                    ii = np.repeat(np.arange(k + 1, nt), 4)
                    r = np.tile(np.arange(4), nt - k - 1)
                    n = len(ii)
                    reqs = np.full((n, 5, 2), -1, dtype=np.int64)
                    reqs[:, 0, 0], reqs[:, 0, 1] = WB + k, MAXB
                    for c in range(4):
                        s_ = sc(4 * ii + r, 4 * k + c)
                        reqs[:, 1 + c, 0], reqs[:, 1 + c, 1] = s_, ver[s_]
                    mark = sc(4 * ii + r, 4 * k)
                    ver[mark] += 1
                    F[4 * ii + r, k] = ver[mark]
                    if sp:
                        key = np.stack([np.full(n, k), np.full(n, 2), ii, r, r * 0, r * 0], 1)
                    elif dl:
                        key = np.stack([ii - 1, np.full(n, k), np.full(n, 3), np.zeros(n, int), r, r * 0], 1)
                    elif rp:
                        key = np.stack([np.full(n, k), np.full(n, 2), ii, np.ones(n, int), r, r * 0], 1)
                    else:
                        key = np.stack([np.full(n, k), np.full(n, 3), np.zeros(n, int), ii, r, r * 0], 1)
                    emit(T_TRSM, ii, np.full(n, k), k, r, 0, 0, mark, reqs, None, "hi", key=key)
                # NEAR(k): the rest of this block's columns, panel k alone
                for j in range(k + 1, k1b):
                    I, J, R, C = subtiles(np.arange(j, nt), np.full(nt - j, j))
                    upd(I, J, R, C, k, 1, True)
            if k1b >= nt:
                continue
            # BULK(b): every later column, panels of the block as one k-run; the next block's columns
            # are high priority (the look-ahead), the rest low
            nk = k1b - k0b
            hi_end = blocks[bi + 1][1]
            for j in range(k1b, nt):
                I, J, R, C = subtiles(np.arange(j, nt), np.full(nt - j, j))
                upd(I, J, R, C, k0b, nk, j < hi_end)
        # ---- flatten: tasks, requirement pairs (compacted), lists
        tasks = np.concatenate([c[0] for c in chunks])
        reqs_all, nreq_all = [], []
        for t, reqs, _ in chunks:
            valid = reqs[:, :, 0] >= 0
            nreq_all.append(valid.sum(1))
            reqs_all.append(reqs[valid])
        nreq = np.concatenate(nreq_all)
        tasks["nreq"] = nreq
        beg = np.zeros(len(tasks), dtype=np.int64)
        beg[1:] = np.cumsum(nreq)[:-1]
        tasks["req_beg"] = beg
        self.tasks = tasks
        self.reqs = np.concatenate(reqs_all).astype(np.int32)
        hk = np.concatenate([k for k, _ in hi_parts])
        hid = np.concatenate([i for _, i in hi_parts])
        order = np.lexsort(tuple(hk[:, q] for q in reversed(range(hk.shape[1]))))
        self.hi = hid[order].astype(np.int32)
        lo_lists: List[np.ndarray] = []
        if lo_parts:
            lx = np.concatenate([np.broadcast_to(x, len(i)) for x, _, i in lo_parts])
            lk = np.concatenate([k for _, k, _ in lo_parts])
            lid = np.concatenate([i for _, _, i in lo_parts])
            for x in range(8):
                m = lx == x
                kk = lk[m]
                o = np.lexsort(tuple(kk[:, q] for q in reversed(range(kk.shape[1]))))
                lo_lists.append(lid[m][o].astype(np.int32))
        else:
            lo_lists = [np.zeros(0, dtype=np.int32) for _ in range(8)]
        self.lo = np.concatenate(lo_lists) if lo_lists else np.zeros(0, dtype=np.int32)
        self.lo_off = np.zeros(9, dtype=np.int64)
        self.lo_off[1:] = np.cumsum([len(x) for x in lo_lists])
        self.final_ver = ver
        self.F = F                                   # strip (I, k) solved: the value of its marker counter
        self.WB = WB
        self.key = np.concatenate(key_parts)         # list order key per task (hi: column-major; lo: its list's)
        self.is_hi = np.zeros(len(tasks), dtype=bool)
        self.is_hi[self.hi] = True
        self.block_of = block_of


# push scheduling classes: 0 POTRF blocks, 1 panel TRSM strips, then the updates by output column j (the step that
# needs them), in at most UPD_BUCKETS buckets
UPD_BUCKETS = int(os.environ.get("DPLASMA_DTR_BUCKETS", "22"))
NCLASS = 2 + UPD_BUCKETS


def queue_edges(tasks, reqs, WB, owner=None, inc_rank=None):
    """Task edges of a requirement-list plan (push scheduling, k_dtr_q).

    Counters live per rank: task t's requirement (c, v) is on rank owner[t]'s counter c; its increment (inc) lands
    on rank inc_rank[t] (its destination for a send).  A requirement on a sub-tile version / strip marker counter
    (c < WB, bumped in emission order, each bump depending on the previous one; a remote strip's arrival counter
    has its single send) names the task of its v-th increment; a W counter (c >= WB: the 16 POTRF blocks of panel
    k, or W_k's 4 arriving column blocks) names all of them.  Returns (ndeps, succ_off, succ)."""
    n = len(tasks)
    owner = np.zeros(n, dtype=np.int64) if owner is None else np.asarray(owner, dtype=np.int64)
    inc_rank = owner if inc_rank is None else np.asarray(inc_rank, dtype=np.int64)
    inc = tasks["inc"].astype(np.int64)
    ncnt = int(max(inc.max(initial=0), int(reqs[:, 0].max()) if len(reqs) else 0)) + 1
    # the increments of every (rank, counter) in emission order
    has = np.nonzero(inc >= 0)[0]
    key = inc_rank[has] * ncnt + inc[has]
    srt = has[np.lexsort((has, key))]
    skey = inc_rank[srt] * ncnt + inc[srt]
    nkey = (int(max(owner.max(initial=0), inc_rank.max(initial=0))) + 1) * ncnt
    cstart = np.searchsorted(skey, np.arange(nkey + 1))
    ccount = np.diff(cstart)
    # requirement records: consumer, (rank, counter), value
    nr = tasks["nreq"].astype(np.int64)
    rt = np.repeat(np.arange(n, dtype=np.int64), nr)
    rb = np.repeat(tasks["req_beg"].astype(np.int64), nr) + (np.arange(int(nr.sum())) - np.repeat(np.cumsum(nr) - nr, nr))
    rc, rv = reqs[rb, 0].astype(np.int64), reqs[rb, 1].astype(np.int64)
    keep = rv > 0
    rt, rc, rv = rt[keep], rc[keep], rv[keep]
    rk = owner[rt] * ncnt + rc
    if np.any(ccount[rk] < rv):
        raise RuntimeError("queue_edges: a requirement names an increment that never happens")
    ver = rc < WB
    cons = [rt[ver]]
    prod = [srt[cstart[rk[ver]] + rv[ver] - 1]]
    w = ~ver
    if w.any():
        m = ccount[rk[w]]
        cons.append(np.repeat(rt[w], m))
        prod.append(srt[np.repeat(cstart[rk[w]], m) + (np.arange(int(m.sum())) - np.repeat(np.cumsum(m) - m, m))])
    cons, prod = np.concatenate(cons), np.concatenate(prod)
    pair = np.unique(prod * n + cons)
    prod, cons = pair // n, pair % n
    ndeps = np.bincount(cons, minlength=n).astype(np.int32)
    succ_off = np.zeros(n + 1, dtype=np.int32)
    succ_off[1:] = np.cumsum(np.bincount(prod, minlength=n))
    succ = cons.astype(np.int32) if len(cons) else np.zeros(1, dtype=np.int32)   # pairs sorted by producer
    return ndeps, succ_off, succ


# weights of the bottom-level priorities (us).  Start: measured mean task durations at one workgroup per CU
# (profiles/r5_dtr_queue.txt: trsm 175, potrf 300); the critical-path tasks are weighted above their mean
# duration -- the sweep in profiles/r5_dtr_bl_weights.txt found trsm 400 / potrf 800 best or tied at 16k, 32k and
# on the emulated 2x4 grid at 64k (75.5 % vs 74.4 %)
TASK_US = {"upd1": 75.0, "upd_k": 65.0, "trsm": 400.0, "potrf": 800.0, "send": 20.0}


def task_weights(tasks):
    # DPLASMA_DTR_BL_W="upd1,upd_k,trsm,potrf" overrides the weights (measurement knob)
    us = dict(TASK_US)
    w = os.environ.get("DPLASMA_DTR_BL_W")
    if w:
        for k_, v in zip(("upd1", "upd_k", "trsm", "potrf"), w.split(",")):
            us[k_] = float(v)
    typ = tasks["type"]
    nk = tasks["nk"].astype(np.float64)
    return np.where(typ == T_UPD, np.maximum(us["upd1"], us["upd_k"] * nk),
                    np.where(typ == T_TRSM, us["trsm"], np.where(typ == T_POTRF, us["potrf"],
                                                                 us["send"]))).astype(np.float64)


def bottom_levels(succ_off, succ, w):
    """Longest weighted path from every task to the end of the factorisation (native, runtime/dag.cpp)."""
    from ..runtime.dag import _lib_rt
    rt = _lib_rt()
    if rt is None or not hasattr(rt, "dag_bottom_level"):
        raise RuntimeError("dtr: the native runtime module (_dplasma_rt) with dag_bottom_level is needed")
    return np.asarray(rt.dag_bottom_level(succ_off, succ, w))


def queue_classes(tasks, nt, succ_off=None, succ=None):
    """(class, XCD) of every task's ready ring.  Class 0: the POTRF blocks (spread over the eight XCDs: the 16
    cooperate and must start together); then every other task by its bottom level -- the longest path of task
    durations from it to the end, the list-scheduling priority of critical-path schedulers -- in UPD_BUCKETS + 1
    buckets, longest first (a tile's chain of deferred updates and the panels behind it rank by what they still
    hold up, not by their output column: ranking by column starved the last columns' update chains, r5_b32).
    XCD: POTRF block % 8, TRSM / sends by tile row, updates by output column (the low lists' L2 locality)."""
    typ = tasks["type"]
    if succ_off is None:
        cls = np.where(typ == T_POTRF, 0, np.where(typ == T_UPD, 2, 1))
    else:
        bl = bottom_levels(succ_off, succ, task_weights(tasks))
        nb_ = NCLASS - 1
        top = max(float(bl.max()), 1e-9)
        cls = np.where(typ == T_POTRF, 0, 1 + np.minimum(nb_ - 1, ((1.0 - bl / top) * nb_).astype(np.int64)))
    xcd = np.where(typ == T_POTRF, tasks["r"] % 8, np.where(typ == T_UPD, tasks["j"] % 8, tasks["i"] % 8))
    return cls.astype(np.int64), xcd.astype(np.int64)


def queue_rings(ring_of, mine, ndeps):
    """One rank's rings: slot offsets per ring (its tasks only) and the initially ready tasks' slots / tails."""
    nring = NCLASS * 8
    cap = np.bincount(ring_of[mine], minlength=nring)
    qbase = np.zeros(nring + 1, dtype=np.int32)
    qbase[1:] = np.cumsum(cap)
    qinit = np.zeros(max(1, int(qbase[-1])), dtype=np.int32)
    tinit = np.zeros(nring, dtype=np.int32)
    for t in np.nonzero(mine & (ndeps == 0))[0]:
        r = ring_of[t]
        qinit[qbase[r] + tinit[r]] = t + 1
        tinit[r] += 1
    return qbase, qinit, tinit


def queue_plan(plan):
    """Push scheduling (k_dtr_q) of a one-process _Plan: queue_edges + one rank's rings.  Returns a dict of arrays:
    ndeps, succ_off, succ, ring_of, qbase, qinit (the initially ready tasks' slots), tinit (initial tails), cls."""
    ndeps, succ_off, succ = queue_edges(plan.tasks, plan.reqs, plan.WB)
    cls, xcd = queue_classes(plan.tasks, plan.nt, succ_off, succ)
    ring_of = (cls * 8 + xcd).astype(np.int32)
    qbase, qinit, tinit = queue_rings(ring_of, np.ones(len(plan.tasks), dtype=bool), ndeps)
    return {"ndeps": ndeps, "succ_off": succ_off, "succ": succ, "ring_of": ring_of, "qbase": qbase,
            "qinit": qinit, "tinit": tinit, "cls": cls}


class ArgsImage:
    """Host image of the kernel's DtrArgs, packed by field name (offsets from dpl_dtr_field: the struct is
    laid out by the device compiler, not mirrored here)."""

    _LL = ("ld", "ncnt", "bw_bpt", "lat_t")
    _INT = ("nt", "nranks", "rank", "epoch", "flags", "dil", "nsteps", "ntask", "nclass")
    _PTR = ("tasks", "reqs", "tab", "xoff", "cur", "hs_off", "scur", "hi", "lo", "vis", "link", "Mw", "Sw", "Lp", "Wp",
            "prog", "info", "trace", "succ_off", "succ", "ring_of", "town", "qbase", "done", "rdy", "probe", "snap")
    _PARR = ("A", "recv", "W", "cnt", "pend", "qctl", "qslot")
    _IARR = ("hi_off", "lo_off")

    def __init__(self, lib):
        self.lib = lib
        f = lambda n: int(lib.dpl_dtr_field(n.encode()))   # noqa: E731
        self.size = f("size")
        if f("task") != TASK_DT.itemsize:
            raise RuntimeError("dtr: DtrTask layout mismatch")
        self.off = {n: f(n) for n in self._LL + self._INT + self._PTR + self._PARR + self._IARR}
        if min(self.off.values()) < 0:
            raise RuntimeError("dtr: the kernel library lacks a DtrArgs field")
        self.maxr = f("MAXR")
        self.pstride = f("PSTRIDE")
        self.buf = bytearray(self.size)

    def set(self, name, v):
        o = self.off[name]
        if name in self._LL:
            struct.pack_into("<q", self.buf, o, int(v))
        elif name in self._INT:
            struct.pack_into("<i", self.buf, o, int(v))
        elif name in self._PTR:
            struct.pack_into("<Q", self.buf, o, int(v or 0))
        elif name in self._PARR:
            vals = list(v) + [0] * (self.maxr - len(v))
            struct.pack_into(f"<{self.maxr}Q", self.buf, o, *[int(x or 0) for x in vals])
        else:
            n = self.maxr + 1 if name == "hi_off" else 9
            vals = list(v) + [v[-1]] * (n - len(v))
            struct.pack_into(f"<{n}i", self.buf, o, *[int(x) for x in vals])


def step_segments(keys_sorted: np.ndarray, order: str, nt: int) -> np.ndarray:
    """Offsets (nt + 1) of the per-step FIFO segments of one rank's high list (sorted by key): with the "step"
    order one segment per panel (key column 0), else one segment holding the whole list."""
    n = len(keys_sorted)
    if order != "step":
        return np.array([0] + [n] * nt, dtype=np.int32)
    steps = keys_sorted[:, 0] if n else np.zeros(0, dtype=np.int64)
    return np.searchsorted(steps, np.arange(nt + 1), side="left").astype(np.int32)


def flags_from_env() -> int:
    # DPLASMA_DTR_STEAL=1: a workgroup whose own XCD list head waits on a dependency takes a ready head of
    # another XCD's list (measurement knob; default: steal only from exhausted lists)
    fl = 1 if os.environ.get("DPLASMA_DTR_STEAL", "0") == "1" else 0
    # DPLASMA_DTR_HOLD="potrf_us,other_us": how long a high-list ticket whose task is not ready yet polls before
    # it runs a low-list task meanwhile (measurement knob; default 50 us for POTRF tickets, 0 for the others)
    # DPLASMA_DTR_SYSACQ=1: system-scope acquire before every task (measurement knob)
    if os.environ.get("DPLASMA_DTR_SYSACQ", "0") == "1":
        fl |= 4
    # DPLASMA_DTR_SYSREL=1: system-scope release after every task (measurement knob)
    if os.environ.get("DPLASMA_DTR_SYSREL", "0") == "1":
        fl |= 8
    # DPLASMA_DTR_WT=1: update / TRSM results stored write-through at system scope (measurement knob)
    if os.environ.get("DPLASMA_DTR_WT", "0") == "1":
        fl |= 16
    # DPLASMA_DTR_STEPW=w: step segments of the high list scanned per claim (1..15; default 8)
    sw = int(os.environ.get("DPLASMA_DTR_STEPW", "0"))
    if sw:
        fl |= (min(15, max(1, sw)) << 24)
    # DPLASMA_DTR_SCANSKIP=0: idle workgroups rescan every ready ring even when no task completed since their last
    # empty scan (measurement knob; default: skip)
    if os.environ.get("DPLASMA_DTR_SCANSKIP", "1") == "0":
        fl |= 32
    # DPLASMA_DTR_NAP=n: the push scheduler's idle back-off cap, n = 2^e sleeps (default 16)
    nap = int(os.environ.get("DPLASMA_DTR_NAP", "0"))
    if nap > 0:
        fl |= (min(7, max(1, nap.bit_length() - 1)) << 28)   # (a signed 32-bit field: e <= 7)
    hold = os.environ.get("DPLASMA_DTR_HOLD")
    if hold:
        hp, ho = (int(x) for x in hold.split(","))
        fl |= (min(255, max(0, ho // 10)) << 8) | (min(255, max(1, hp // 10)) << 16)
    return fl


def tile_offsets(A, nt):
    """nt x nt table (i + j nt) of A's tile element offsets for i >= j (local tiles only), -1 elsewhere."""
    tab = np.full(nt * nt, -1, dtype=np.int64)
    for j in range(nt):
        for i in range(j, nt):
            if A.is_local(i, j):
                tab[i + j * nt] = A.offset(i, j)
    return tab


class PotrfScratch:
    """Per-panel POTRF workspaces of one launch (indexed by panel: disjoint across the ranks of an emulation)."""

    def __init__(self, nt, dev, pstride):
        self.Mw = torch.zeros(nt * MAXB * BLK, dtype=torch.float64, device=dev)
        self.Sw = torch.zeros(nt * MAXB * RB, dtype=torch.float64, device=dev)
        self.Lp = torch.zeros(nt * MAXB * MAXB * BLK, dtype=torch.float64, device=dev)
        self.Wp = torch.zeros(nt * MAXB * MAXB * BLK, dtype=torch.float64, device=dev)
        self.prog = torch.zeros(nt * 2 * MAXB * pstride, dtype=torch.int32, device=dev)

    def fill(self, img):
        for n in ("Mw", "Sw", "Lp", "Wp", "prog"):
            img.set(n, getattr(self, n).data_ptr())


_PLANS = {}


def _plan_cache_path(nt, D, lo_order, min_tiles, head):
    """On-disk cache of a one-process plan and its push-scheduling arrays (the 64k plan: 1.57 M tasks, 13 M edges,
    ~6.5 s of host time to build).  Keyed by the plan parameters, the priority knobs and a hash of this module's
    source, so an edited planner never reads an old plan.  DPLASMA_DTR_PLAN_CACHE: directory (default
    ~/.cache/dplasma_amd), "0" disables."""
    import hashlib
    d = os.environ.get("DPLASMA_DTR_PLAN_CACHE", os.path.join(os.path.expanduser("~"), ".cache", "dplasma_amd"))
    if d == "0" or nt < 48:   # (small plans build in well under a second)
        return None
    with open(__file__, "rb") as f:
        src = hashlib.sha1(f.read()).hexdigest()[:12]
    knobs = f"{UPD_BUCKETS}_{os.environ.get('DPLASMA_DTR_BL_W', '')}"
    tag = hashlib.sha1(f"{nt}_{D}_{lo_order}_{min_tiles}_{head}_{knobs}_{src}".encode()).hexdigest()[:16]
    return os.path.join(d, f"dtr_plan_{nt}_{tag}.npz")


_PLAN_ARR = ("reqs", "hi", "lo", "lo_off", "final_ver", "F", "key", "is_hi", "block_of")
_PLAN_INT = ("nt", "S", "D", "ncnt", "WB")


def _plan_load(path):
    """A cached plan (None when absent or unreadable); plain arrays only (allow_pickle=False)."""
    try:
        with np.load(path, allow_pickle=False) as z:
            pl = _Plan.__new__(_Plan)
            pl.tasks = z["tasks"].view(TASK_DT).reshape(-1)
            for n in _PLAN_ARR:
                setattr(pl, n, z[n])
            for n in _PLAN_INT:
                setattr(pl, n, int(z[n]))
            pl.order = str(z["order"])
            pl.blocks = [tuple(int(x) for x in b) for b in z["blocks"]]
            pl._queue = {n[2:]: z[n] for n in z.files if n.startswith("q_")}
        return pl
    except (OSError, KeyError, ValueError):
        return None


def _plan_save(path, pl):
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        arrs = {n: getattr(pl, n) for n in _PLAN_ARR}
        arrs.update({n: np.int64(getattr(pl, n)) for n in _PLAN_INT})
        arrs["tasks"] = pl.tasks.view(np.uint8)
        arrs["order"] = np.array(pl.order)
        arrs["blocks"] = np.array(pl.blocks, dtype=np.int64).reshape(-1, 2)
        arrs.update({f"q_{n}": v for n, v in pl._queue.items()})
        tmp = f"{path}.{os.getpid()}.tmp.npz"
        np.savez(tmp, **arrs)
        os.replace(tmp, path)   # (atomic: a concurrent reader sees the old file or the whole new one)
    except OSError:
        pass


def _get_plan(nt, D, lo_order, min_tiles, head):
    key = (nt, D, lo_order, min_tiles, head)
    plan = _PLANS.get(key)
    if plan is not None:
        return plan
    path = _plan_cache_path(nt, D, lo_order, min_tiles, head)
    plan = _plan_load(path) if path and os.path.exists(path) else None
    if plan is None:
        plan = _Plan(nt, D, lo_order, min_tiles, head)
        if path:
            plan._queue = queue_plan(plan)
            _plan_save(path, plan)
    _PLANS[key] = plan
    return plan


def potrf_dtr_New(ctx, uplo: int, A, info_out=None) -> Taskpool:
    from ..ops import _lib
    if not supported(ctx, uplo, A):
        raise ValueError("potrf_dtr: one process, lower, fp64, NB = 512, N a multiple of 512, GPU")
    lib = _lib.load()
    img = ArgsImage(lib)
    PST = img.pstride
    nt = A.nt
    D = max(1, int(os.environ.get("DPLASMA_DTR_DEFER", "4")))
    lo_order = os.environ.get("DPLASMA_DTR_LO_ORDER", "column")
    min_tiles = int(os.environ.get("DPLASMA_DTR_DEFER_MIN_TILES", "0"))
    head = _head_env()
    plan = _get_plan(nt, D, lo_order, min_tiles, head)
    dev = A.device
    tp = Taskpool("potrf", ctx)
    tp.flops = flops(A.prec, "potrf", A.n)
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    tp.info = info

    def up(x):
        return torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    tasks_d = up(plan.tasks.view(np.uint8))
    reqs_d = up(plan.reqs)
    hi_d = up(plan.hi)
    lo_d = up(plan.lo if len(plan.lo) else np.zeros(1, dtype=np.int32))
    si, sj = _strides(A)
    tab = np.full(nt * nt, -1, dtype=np.int64)
    for j in range(nt):
        tab[j * nt + j: (j + 1) * nt] = np.arange(j, nt, dtype=np.int64) * si + j * sj
    tab_d = up(tab)
    cnt = torch.zeros(plan.ncnt, dtype=torch.int32, device=dev)
    cur = torch.zeros((img.maxr + 8) * PST, dtype=torch.int32, device=dev)
    hs = step_segments(plan.key[plan.hi], plan.order, nt)
    hs_d = up(hs)
    scur = torch.zeros(nt * PST, dtype=torch.int32, device=dev)
    # per-panel workspaces (HBM is plentiful: ~6 MB per panel, nothing recycled, no WAR edges)
    W = torch.zeros(nt * NBT * NBT, dtype=torch.float64, device=dev)
    scr = PotrfScratch(nt, dev, PST)
    img.set("ld", A.ld)
    img.set("nt", nt)
    img.set("nranks", 1)
    img.set("rank", 0)
    img.set("dil", 1)
    img.set("ncnt", plan.ncnt)
    img.set("tasks", tasks_d.data_ptr())
    img.set("reqs", reqs_d.data_ptr())
    img.set("tab", tab_d.data_ptr())
    img.set("cur", cur.data_ptr())
    img.set("nsteps", nt)
    img.set("hs_off", hs_d.data_ptr())
    img.set("scur", scur.data_ptr())
    img.set("hi", hi_d.data_ptr())
    img.set("hi_off", [0, len(plan.hi)])
    img.set("lo", lo_d.data_ptr())
    img.set("lo_off", plan.lo_off)
    img.set("A", [A.data.data_ptr()])
    img.set("W", [W.data_ptr()])
    img.set("cnt", [cnt.data_ptr()])
    scr.fill(img)
    img.set("info", info.data_ptr())
    img.set("flags", flags_from_env())
    # DPLASMA_DTR_TRACE=1: per-task {start, end, workgroup << 8 | xcd} (s_memrealtime, 100 MHz) in tp.dtr_trace
    trace = None
    if os.environ.get("DPLASMA_DTR_TRACE", "0") == "1":
        # + the POTRF blocks' phase stamps (dtr.hip run_potrf: 64 per block, nt x 16 blocks)
        trace = torch.zeros(4 * len(plan.tasks) + nt * MAXB * 64, dtype=torch.int64, device=dev)
        img.set("trace", trace.data_ptr())
    tp.dtr_trace = trace
    # DPLASMA_DTR_PROBE=1: the strip-hazard probe of the diagonal-tile updates (tp.dtr_probe; dtr.hip probe_strip)
    probe = None
    if os.environ.get("DPLASMA_DTR_PROBE", "0") == "1":
        probe = torch.zeros(8 + 20 * nt * nt + 8 * 4096, dtype=torch.int64, device=dev)
        img.set("probe", probe.data_ptr())
    tp.dtr_probe = probe
    snap = None
    if os.environ.get("DPLASMA_DTR_SNAP", "0") == "1":
        snap = torch.zeros(nt * NBT * NBT, dtype=torch.float64, device=dev)
        img.set("snap", snap.data_ptr())
    tp.dtr_snap = snap
    nbytes = img.size
    host = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    hosts = [[host, None], [torch.empty(nbytes, dtype=torch.uint8).pin_memory(), None]]
    args_d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    state = {"epoch": 0}
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    # one workgroup per CU by default: faster than two with the push scheduler at 16k / 32k / 64k (48.0 / 61.8 / 64.9
    # vs 28.4 / 55.8 / 62.6 TF/s).  Two per CU (DPLASMA_DTR_WG=512) are correct since round 6: the intermittent wrong
    # factor of round 5 was an inline-asm store in the tile POTRF (profiles/r6_dtr_coresidency_rootcause.txt)
    nwg = int(os.environ.get("DPLASMA_DTR_WG", ncu))
    # progress needs a workgroup on every XCD (a low list is another XCD's to steal only once that XCD's
    # own list is exhausted) and the 16 cooperating POTRF workgroups co-resident: at least 64 of them
    nwg = max(64, min(nwg, 2 * ncu))
    if nwg > ncu:
        # two per CU: the idle scan skip was only exercised at one per CU (a box was lost during the first 512-
        # workgroup run with it, cause not established), so this configuration keeps the full rescan it was
        # validated with (0 / 100 wrong factors, profiles/r6_dtr_coresidency_rootcause.txt)
        img.set("flags", flags_from_env() | 32)
    # scheduling: "queue" (default) -- push scheduling, a task is pushed into its priority class's ready ring by
    # the completion of its last predecessor (k_dtr_q, queue_plan); "lists" -- the static high / low lists with
    # version-counter readiness (k_dtr_potrf)
    sched = os.environ.get("DPLASMA_DTR_SCHED", "queue")
    if sched not in ("queue", "lists"):
        raise ValueError("DPLASMA_DTR_SCHED must be queue or lists")
    qk = None
    if sched == "queue":
        qp = getattr(plan, "_queue", None)
        if qp is None:
            qp = plan._queue = queue_plan(plan)
        nring = NCLASS * 8
        qctl_init = torch.zeros(2 * nring * PST, dtype=torch.int32)
        qctl_init.view(nring, 2, PST)[:, 1, 0] = torch.from_numpy(qp["tinit"])
        qk = {"pend0": up(qp["ndeps"]), "pend": torch.empty(len(qp["ndeps"]), dtype=torch.int32, device=dev),
              "succ_off": up(qp["succ_off"]), "succ": up(qp["succ"]), "ring_of": up(qp["ring_of"]),
              "qbase": up(qp["qbase"]), "qctl0": qctl_init.to(dev), "qctl": torch.empty(2 * nring * PST, dtype=torch.int32,
                                                                                          device=dev),
              "qslot0": up(qp["qinit"]), "qslot": torch.empty(len(qp["qinit"]), dtype=torch.int32, device=dev),
              "done": torch.zeros(1, dtype=torch.int32, device=dev)}
        img.set("ntask", len(plan.tasks))
        img.set("nclass", NCLASS)
        for f in ("succ_off", "succ", "ring_of", "qbase", "done"):
            img.set(f, qk[f].data_ptr())
        for f in ("pend", "qctl", "qslot"):
            img.set(f, [qk[f].data_ptr()])
    tp._keep = (tasks_d, reqs_d, hi_d, lo_d, tab_d, cnt, cur, hs_d, scur, W, scr, hosts, args_d, qk, probe, snap)
    tp.dtr_plan = plan
    tp.dtr_sched = sched

    def f_run():
        state["epoch"] = state["epoch"] % ((1 << 25) - 1) + 1
        img.set("epoch", state["epoch"])
        # a pinned staging buffer per run slot: a non-blocking copy still pending from an earlier run (runs
        # issued back to back, no host sync between them) must not see this run's epoch
        slot = hosts[state["epoch"] % len(hosts)]
        if slot[1] is not None:
            slot[1].synchronize()
        slot[0].numpy()[:] = np.frombuffer(bytes(img.buf), dtype=np.uint8)
        args_d.copy_(slot[0], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        slot[1] = ev
        if qk is not None:
            qk["pend"].copy_(qk["pend0"])
            qk["qctl"].copy_(qk["qctl0"])
            qk["qslot"].copy_(qk["qslot0"])
            qk["done"].zero_()
            _lib.check(lib.dpl_dtr_potrf_q(args_d.data_ptr(), nwg, _lib.stream_ptr()), "dtr_potrf_q")
            return
        cnt.zero_()
        cur.zero_()
        scur.zero_()
        _lib.check(lib.dpl_dtr_potrf(args_d.data_ptr(), nwg, _lib.stream_ptr()), "dtr_potrf")

    tp.task("DTR_POTRF", "update", f_run)

    def _done():
        r = int(info.item())
        if r < 0:
            raise RuntimeError(f"potrf: device task runtime failure (info {r})")
        if info_out is not None:
            info_out[0] = r
        return r
    tp.on_complete(_done)
    return tp.finish_build()
