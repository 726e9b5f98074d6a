"""Distributed device task runtime Cholesky: every rank of a P x Q grid runs the DTR on its own tiles.

The reference schedules the Cholesky PTG on every rank with priorities, and a task whose input is a
remote tile waits for the remote-dependency engine to deliver it (``src/zpotrf_L.jdf:58-69``
priorities, ``high_priority`` at ``:93, 194, 306``; the flows ``A <- A potrf_ztrsm(k, m)`` of the
update classes cross ranks).  Here the same happens inside ONE persistent launch per rank
(``csrc/kernels/dtr.hip``): a remote panel strip is a task *requirement* -- an arrival counter on the
consumer rank -- and the producer's ``SEND`` task (high priority, right behind the ``TRSM`` that
solved the strip) stores the strip into the consumer's receive buffer and bumps that counter; no
separate transport kernel competes for the CUs the persistent kernel holds.

Plan (this module), from the one-process plan of ``models/potrf_dtr.py``:

* every task runs on the owner of the tile it writes (``UPD(i, j, ..)`` and ``TRSM(i, k, r)`` on
  owner(i, j) / owner(i, k), ``POTRF(k, b)`` on owner(k, k));
* an update's requirement on a strip of a remote panel tile becomes "arrival counter >= 1" on its
  rank; a ``SEND(i, k, r, dest)`` task per (strip, consumer rank) requires the strip solved on the
  producer and bumps the consumer's counter (same counter index on every rank: the strip's marker);
* a ``TRSM(i, k, r)`` away from owner(k, k) needs ``W_k = L_kk^-T``: ``SENDW(k, c, dest)`` tasks copy
  its four 128-column blocks (upper triangle only) into the consumer's ``W``; the consumer's TRSM
  requires 4 arrivals instead of the 16 POTRF block columns;
* every remote tile a rank reads gets its own receive slot (HBM is plentiful: ~0.75 nt^2 / 2 / (P Q)
  tiles per rank, nothing recycled, so no write-after-read hazards);
* lists: each rank's high list is the one-process high order restricted to its tasks, with ``SEND``
  right behind its ``TRSM`` and ``SENDW`` right behind POTRF(k); its low tasks are split over the
  XCDs it runs on by column, each list in the one-process low order.  Every list is a subsequence of
  the one-process topological order extended by the sends, so the earliest unfinished task of that
  order is always claimable on its rank: the distributed schedule cannot deadlock either
  (``tests/test_potrf_dtr.py`` runs the protocol over ranks with random completion orders).

Two execution modes share the kernel: one process per GPU (``rank >= 0``; peers' receive buffers,
``W`` and counters IPC-mapped, system-scope stores + release) and the *emulation* of a grid on one
GPU (``rank = -1``): each XCD is a rank's "GPU" (8 ranks: one XCD each), the sends are copies inside
HBM, and time is dilated by the number of ranks -- every task's completion becomes visible
(nranks - 1) x its duration late and a send lands ``nranks x (lat + bytes / bw)`` after its link
(one per ordered rank pair, FIFO) frees up -- so the launch's span / nranks models the P x Q run
(``tools/emulate_potrf.py``).
"""
from __future__ import annotations

import numpy as np

from . import potrf_dtr as D

T_UPD, T_TRSM, T_POTRF = D.T_UPD, D.T_TRSM, D.T_POTRF
T_SEND, T_SENDW = 3, 4
NBT, MAXB = D.NBT, D.MAXB
STRIP = 128 * NBT                     # elements of a 128-row strip of a 512 x 512 tile


def _unique_pairs(a, b):
    """np.unique(np.stack([a, b], 1), axis=0) for non-negative integer columns, through one 1-D key (the row-wise
    unique sorts structured rows: 14 s of a 64k 2 x 4 plan)."""
    a, b = np.asarray(a, dtype=np.int64), np.asarray(b, dtype=np.int64)
    m = int(b.max()) + 1 if len(b) else 1
    k = np.unique(a * m + b)
    return np.stack([k // m, k % m], 1)


class DistPlan:
    """Per-rank task lists, requirement targets, sends and receive slots of a P x Q grid."""

    def __init__(self, nt: int, Dd: int, P: int, Q: int, lo_order: str = None, min_tiles: int = None,
                 base: "D._Plan" = None):
        base = base or D._Plan(nt, Dd, lo_order, min_tiles)
        self.base, self.nt, self.P, self.Q, self.nranks = base, nt, P, Q, P * Q
        S, WB = base.S, base.WB
        self.S, self.WB, self.ncnt = S, WB, base.ncnt
        tasks = base.tasks.copy()
        reqs = base.reqs.copy()
        ntask0 = len(tasks)
        own = self._owner(tasks["i"].astype(np.int64), tasks["j"].astype(np.int64))
        # ---- requirement translation (remote strips / remote W_k)
        nreq = tasks["nreq"].astype(np.int64)
        rtask = np.repeat(np.arange(ntask0), nreq)
        rpos = np.arange(len(reqs)) - np.repeat(tasks["req_beg"].astype(np.int64), nreq)
        ttype = tasks["type"][rtask]
        towner = own[rtask]
        idx = reqs[:, 0].astype(np.int64)
        strip_req = (ttype == T_UPD) & (rpos >= 1)
        I, J = idx % S, idx // S
        powner = self._owner(I // 4, J // 4)
        remote_strip = strip_req & (powner != towner)
        # consumers of remote strips: unique (counter, consumer rank)
        cons = _unique_pairs(idx[remote_strip], towner[remote_strip]) if remote_strip.any() \
            else np.zeros((0, 2), dtype=np.int64)
        reqs[remote_strip, 1] = 1
        w_req = (ttype == T_TRSM) & (rpos == 0)
        kW = idx - WB
        wowner = self._owner(kW, kW)
        remote_w = w_req & (wowner != towner)
        wcons = _unique_pairs(kW[remote_w], towner[remote_w]) if remote_w.any() \
            else np.zeros((0, 2), dtype=np.int64)
        reqs[remote_w, 1] = 4
        # ---- send tasks
        ns, nw = len(cons), 4 * len(wcons)
        st = np.zeros(ns + nw, dtype=D.TASK_DT)
        sreq = np.zeros((ns + nw, 2), dtype=np.int64)
        keys = np.zeros((ns + nw, 6), dtype=np.int64)
        sown = np.zeros(ns + nw, dtype=np.int64)
        if ns:
            c_idx, dest = cons[:, 0], cons[:, 1]
            Is, ks = c_idx % S, c_idx // S // 4
            st["type"][:ns], st["i"][:ns], st["j"][:ns], st["k0"][:ns] = T_SEND, Is // 4, dest, ks
            st["r"][:ns], st["inc"][:ns] = Is % 4, c_idx
            sreq[:ns, 0] = c_idx
            sreq[:ns, 1] = base.F[Is, ks]            # the strip's "solved" marker value on the producer
            if base.order == "deadline":
                keys[:ns] = np.stack([Is // 4 - 1, ks, np.full(ns, 3), np.zeros(ns, int), Is % 4, 1 + dest], 1)
            elif base.order == "rowpipe":
                keys[:ns] = np.stack([ks, np.full(ns, 2), Is // 4, np.ones(ns, int), Is % 4, 1 + dest], 1)
            elif base.order == "step":
                keys[:ns] = np.stack([ks, np.full(ns, 2), Is // 4, Is % 4, 1 + dest, np.zeros(ns, int)], 1)
            else:
                keys[:ns] = np.stack([ks, np.full(ns, 3), np.zeros(ns, int), Is // 4, Is % 4, 1 + dest], 1)
            sown[:ns] = self._owner(Is // 4, ks)
        if nw:
            kk = np.repeat(wcons[:, 0], 4)
            dest = np.repeat(wcons[:, 1], 4)
            cb = np.tile(np.arange(4), len(wcons))
            sl = slice(ns, ns + nw)
            st["type"][sl], st["i"][sl], st["j"][sl], st["k0"][sl] = T_SENDW, kk, dest, kk
            st["r"][sl], st["inc"][sl] = cb, WB + kk
            sreq[sl, 0], sreq[sl, 1] = WB + kk, MAXB
            if base.order == "deadline":
                keys[sl] = np.stack([kk, kk, np.ones(nw, int), np.ones(nw, int), MAXB + cb, dest], 1)
            elif base.order == "step":
                keys[sl] = np.stack([kk, np.ones(nw, int), np.zeros(nw, int), np.zeros(nw, int), cb, dest], 1)
            else:
                keys[sl] = np.stack([kk, np.ones(nw, int), np.zeros(nw, int), MAXB + cb, dest, np.zeros(nw, int)], 1)
            sown[sl] = self._owner(kk, kk)
        st["nreq"] = 1
        st["req_beg"] = len(reqs) + np.arange(ns + nw)
        self.tasks = np.concatenate([tasks, st])
        self.reqs = np.concatenate([reqs, sreq]).astype(np.int32)
        self.owner = np.concatenate([own, sown])
        self.key = np.concatenate([base.key, keys])
        self.is_hi = np.concatenate([base.is_hi, np.ones(ns + nw, dtype=bool)])
        self.nsend, self.nsendw = ns, nw
        # ---- receive slots: every remote panel tile a rank reads
        self.recv_tiles = []
        self.recv_slot = []
        for r in range(self.nranks):
            sel = cons[:, 1] == r if ns else np.zeros(0, dtype=bool)
            tl = _unique_pairs((cons[sel, 0] % S) // 4, cons[sel, 0] // S // 4) \
                if ns and sel.any() else np.zeros((0, 2), dtype=np.int64)
            self.recv_tiles.append(tl)
            self.recv_slot.append({(int(i), int(k)): q for q, (i, k) in enumerate(tl)})
        # send destinations: element offset in the destination's receive buffer (SEND) or W (SENDW)
        self.xoff = np.zeros(len(self.tasks), dtype=np.int64)
        for q in range(ns):
            t = self.tasks[ntask0 + q]
            slot = self.recv_slot[int(t["j"])][(int(t["i"]), int(t["k0"]))]
            self.xoff[ntask0 + q] = slot * NBT * NBT + 128 * int(t["r"])
        if nw:
            tw = self.tasks[ntask0 + ns:]
            self.xoff[ntask0 + ns:] = tw["k0"].astype(np.int64) * NBT * NBT + tw["r"].astype(np.int64) * 128 * NBT

    def queue(self):
        """Push scheduling over the grid (k_dtr_q in process mode): global task edges -- a send's successors live
        on its destination rank, whose pending counts and rings it updates through the IPC mapping -- and every
        rank's rings (cached)."""
        q = getattr(self, "_queue", None)
        if q is not None:
            return q
        typ = self.tasks["type"]
        inc_rank = np.where((typ == T_SEND) | (typ == T_SENDW), self.tasks["j"].astype(np.int64), self.owner)
        ndeps, succ_off, succ = D.queue_edges(self.tasks, self.reqs, self.WB, self.owner, inc_rank)
        cls, xcd = D.queue_classes(self.tasks, self.nt, succ_off, succ)
        ring_of = (cls * 8 + xcd).astype(np.int32)
        qbase, qinit, tinit, nown = [], [], [], []
        for r in range(self.nranks):
            mine = self.owner == r
            b, qi, ti = D.queue_rings(ring_of, mine, ndeps)
            qbase.append(b)
            qinit.append(qi)
            tinit.append(ti)
            nown.append(int(mine.sum()))
        self._queue = q = {"ndeps": ndeps, "succ_off": succ_off, "succ": succ, "ring_of": ring_of, "cls": cls,
                           "town": self.owner.astype(np.int32), "qbase": np.concatenate(qbase), "qinit": qinit,
                           "tinit": tinit, "nown": nown}
        return q

    def _owner(self, i, j):
        return (np.asarray(i) % self.P) * self.Q + (np.asarray(j) % self.Q)

    # ------------------------------------------------------------------ lists
    def lists(self, xcds_of: dict):
        """xcds_of: rank -> the XCD ids its workgroups run on (a process: all 8; the emulation: its own).
        Returns (hi, hi_off[nranks + 1], lo, lo_off[9]): each rank's high list (in the one-process high order
        with the sends inserted) and one low list per XCD (the rank's low tasks by column, one-process order)."""
        hi_parts, hi_off = [], [0]
        lo_lists = [np.zeros(0, dtype=np.int32) for _ in range(8)]
        nr = self.nranks
        for r in range(nr):
            mine = self.owner == r
            h = np.nonzero(mine & self.is_hi)[0]
            kk = self.key[h]
            o = np.lexsort(tuple([h] + [kk[:, q] for q in reversed(range(6))]))
            hi_parts.append(h[o].astype(np.int32))
            hi_off.append(hi_off[-1] + len(h))
            xs = list(xcds_of.get(r, []))
            if not xs:
                continue
            lo = np.nonzero(mine & ~self.is_hi)[0]
            kk = self.key[lo]
            o = np.lexsort(tuple([lo] + [kk[:, q] for q in reversed(range(6))]))
            lo = lo[o]
            col = self.tasks["j"][lo].astype(np.int64)
            pick = (col // self.Q) % len(xs)
            for q, x in enumerate(xs):
                lo_lists[x] = np.concatenate([lo_lists[x], lo[pick == q].astype(np.int32)])
        self.hs_off = np.concatenate([D.step_segments(self.key[h], self.base.order, self.nt) for h in hi_parts])
        hi = np.concatenate(hi_parts) if hi_parts else np.zeros(0, dtype=np.int32)
        lo_off = np.zeros(9, dtype=np.int64)
        lo_off[1:] = np.cumsum([len(x) for x in lo_lists])
        return hi, np.asarray(hi_off + [hi_off[-1]] * (8 - nr), dtype=np.int64), np.concatenate(lo_lists), lo_off

    def recv_elems(self, r: int) -> int:
        return max(1, len(self.recv_tiles[r])) * NBT * NBT

    def tile_table(self, r: int, tile_off, recv_base_off: int) -> np.ndarray:
        """nt x nt element offsets (relative to rank r's A base; column-major by (i, j)): r's local tiles
        (tile_off(i, j)) and its received copies (recv_base_off + slot * NB^2); -1 elsewhere."""
        nt = self.nt
        tab = np.full(nt * nt, -1, dtype=np.int64)
        for j in range(nt):
            for i in range(j, nt):
                if self._owner(i, j) == r:
                    tab[i + j * nt] = tile_off(i, j)
        for (i, k), q in self.recv_slot[r].items():
            tab[i + k * nt] = recv_base_off + q * NBT * NBT
        return tab


# ------------------------------------------------------------------------------------------ emulation
class Emulation:
    """A P x Q grid's DTR Cholesky emulated on ONE GPU (see the module docstring): every rank's tiles in its
    own TILE-storage descriptor, receive buffer, W and counters; one launch of 2 x #CUs workgroups whose
    XCD picks their rank; time dilated by P Q.  ``run()`` returns the launch span (s); the modelled P x Q
    time is span / (P Q)."""

    def __init__(self, ctx, N: int, P: int, Q: int, bw_gbs: float = 50.0, lat_us: float = 10.0, Dd: int = None,
                 seed: int = 3872, trace: bool = False, order: str = None):
        import os

        import torch

        from .. import descriptor as dsc
        from ..ops import _lib
        nr = P * Q
        if 8 % nr or N % NBT:
            raise ValueError("emulation: P Q must divide 8 (one or more XCDs per rank) and N a multiple of 512")
        self.ctx, self.N, self.P, self.Q, self.nr = ctx, N, P, Q, nr
        nt = N // NBT
        Dd = Dd or max(1, int(os.environ.get("DPLASMA_DTR_DEFER", "4")))
        self.plan = plan = DistPlan(nt, Dd, P, Q, lo_order=order or os.environ.get("DPLASMA_DTR_LO_ORDER", "step"))
        lib = _lib.load()
        self.lib = lib
        img = D.ArgsImage(lib)
        self.img = img
        dev = ctx.device
        X = 8 // nr
        hi, hi_off, lo, lo_off = plan.lists({r: list(range(r * X, (r + 1) * X)) for r in range(nr)})

        def up(x):
            return torch.from_numpy(np.ascontiguousarray(x)).to(dev)
        # per-rank storage: the P x Q block-cyclic descriptors of rank r (TILE storage, 512 x 512 tiles)
        self.A = [dsc.TiledMatrix(torch.float64, NBT, NBT, N, N, P=P, Q=Q, rank=r, device=dev) for r in range(nr)]
        from .aux import plghe
        for Ar in self.A:
            plghe(ctx, float(N), 123, Ar, seed)      # dplasmaUpperLower: bit-identical for any distribution
        self.A0 = [Ar.data.clone() for Ar in self.A]
        self.recv = [torch.zeros(plan.recv_elems(r), dtype=torch.float64, device=dev) for r in range(nr)]
        self.W = [torch.zeros(nt * NBT * NBT, dtype=torch.float64, device=dev) for _ in range(nr)]
        self.cnt = torch.zeros(nr * plan.ncnt, dtype=torch.int32, device=dev)
        self.vis = torch.zeros(nr * plan.ncnt, dtype=torch.int64, device=dev)
        self.link = torch.zeros(img.maxr * img.maxr, dtype=torch.int64, device=dev)
        self.cur = torch.zeros((img.maxr + 8) * img.pstride, dtype=torch.int32, device=dev)
        self.hs_d = up(plan.hs_off)
        self.scur = torch.zeros(nr * nt * img.pstride, dtype=torch.int32, device=dev)
        tabs = []
        for r in range(nr):
            rb = (self.recv[r].data_ptr() - self.A[r].data.data_ptr())
            assert rb % 8 == 0
            tabs.append(plan.tile_table(r, self.A[r].offset, rb // 8))
        self.tab_d = up(np.concatenate(tabs))
        self.tasks_d = up(plan.tasks.view(np.uint8))
        self.reqs_d = up(plan.reqs)
        self.xoff_d = up(plan.xoff)
        self.hi_d = up(hi if len(hi) else np.zeros(1, dtype=np.int32))
        self.lo_d = up(lo if len(lo) else np.zeros(1, dtype=np.int32))
        self.info = torch.zeros(1, dtype=torch.int32, device=dev)
        self.scr = D.PotrfScratch(nt, dev, img.pstride)
        # (+ the POTRF blocks' phase stamps, dtr.hip run_potrf)
        self.trace = (torch.zeros(4 * len(plan.tasks) + nt * D.MAXB * 64, dtype=torch.int64, device=dev)
                      if trace else None)
        img.set("ld", NBT)
        img.set("nt", nt)
        img.set("nranks", nr)
        img.set("rank", -1)
        img.set("dil", nr)
        img.set("ncnt", plan.ncnt)
        img.set("tasks", self.tasks_d.data_ptr())
        img.set("reqs", self.reqs_d.data_ptr())
        img.set("tab", self.tab_d.data_ptr())
        img.set("xoff", self.xoff_d.data_ptr())
        img.set("cur", self.cur.data_ptr())
        img.set("nsteps", nt)
        img.set("hs_off", self.hs_d.data_ptr())
        img.set("scur", self.scur.data_ptr())
        img.set("hi", self.hi_d.data_ptr())
        img.set("hi_off", hi_off)
        img.set("lo", self.lo_d.data_ptr())
        img.set("lo_off", lo_off)
        img.set("A", [a.data.data_ptr() for a in self.A])
        img.set("recv", [b.data_ptr() for b in self.recv])
        img.set("W", [w.data_ptr() for w in self.W])
        img.set("cnt", [self.cnt.data_ptr() + 4 * r * plan.ncnt for r in range(nr)])
        img.set("vis", self.vis.data_ptr())
        img.set("link", self.link.data_ptr())
        img.set("bw_bpt", max(1, int(round(bw_gbs * 10))))
        img.set("lat_t", int(round(lat_us * 100)))
        self.scr.fill(img)
        img.set("info", self.info.data_ptr())
        img.set("flags", D.flags_from_env())
        if trace:
            img.set("trace", self.trace.data_ptr())
        # scheduling (DPLASMA_DTR_SCHED): "queue" -- push scheduling (k_dtr_q; every rank's rings on its own XCDs,
        # a successor's visibility the latest of its predecessors' dilated completions), "lists" -- k_dtr_potrf
        self.sched = os.environ.get("DPLASMA_DTR_SCHED", "queue")
        self.qk = None
        if self.sched == "queue":
            qp = plan.queue()
            nring = D.NCLASS * 8
            own = plan.owner.astype(np.int64)
            xr = (own * X + (qp["ring_of"] % 8) % X)                     # the owner rank's XCDs
            ring_of = ((qp["ring_of"] // 8) * 8 + xr).astype(np.int32)
            bases, qctl0, qslot0 = [], [], []
            for r in range(nr):
                b, qi, ti = D.queue_rings(ring_of, own == r, qp["ndeps"])
                bases.append(b)
                c0 = torch.zeros(2 * nring * img.pstride, dtype=torch.int32)
                c0.view(nring, 2, img.pstride)[:, 1, 0] = torch.from_numpy(ti)
                qctl0.append(c0.to(dev))
                qslot0.append(up(qi))
            self.qk = qk = {"pend0": up(qp["ndeps"]), "qctl0": qctl0, "qslot0": qslot0,
                            "pend": [torch.empty(len(plan.tasks), dtype=torch.int32, device=dev) for _ in range(nr)],
                            "qctl": [torch.empty_like(c) for c in qctl0], "qslot": [torch.empty_like(q_) for q_ in qslot0],
                            "succ_off": up(qp["succ_off"]), "succ": up(qp["succ"]), "ring_of": up(ring_of),
                            "town": up(qp["town"]), "qbase": up(np.concatenate(bases)),
                            "done": torch.zeros(1, dtype=torch.int32, device=dev),
                            "rdy": torch.zeros(len(plan.tasks), dtype=torch.int64, device=dev)}
            img.set("ntask", len(plan.tasks))
            img.set("nclass", D.NCLASS)
            for f in ("succ_off", "succ", "ring_of", "town", "qbase", "done", "rdy"):
                img.set(f, qk[f].data_ptr())
            for f in ("pend", "qctl", "qslot"):
                img.set(f, [t_.data_ptr() for t_ in qk[f]])
        self.args_d = torch.empty(img.size, dtype=torch.uint8, device=dev)
        self.epoch = 0
        ncu = torch.cuda.get_device_properties(dev).multi_processor_count
        # one workgroup per CU, as the process mode and the one-GPU DTR (the round-5 figures were taken with
        # DPLASMA_DTR_WG=256; two per CU models the grid ~2x slower at 32k: 22 % vs 39 %, r6_b39 / r6_b41)
        self.nwg = int(os.environ.get("DPLASMA_DTR_WG", ncu))

    def reset(self):
        for Ar, a0 in zip(self.A, self.A0):
            Ar.data.copy_(a0)

    def run(self) -> float:
        import time

        import torch

        from ..ops import _lib
        self.epoch = self.epoch % ((1 << 25) - 1) + 1
        self.img.set("epoch", self.epoch)
        self.args_d.copy_(torch.frombuffer(bytearray(self.img.buf), dtype=torch.uint8))
        for t in (self.cnt, self.vis, self.link, self.cur, self.scur, self.info):
            t.zero_()
        qk = self.qk
        if qk is not None:
            for r in range(self.nr):
                qk["pend"][r].copy_(qk["pend0"])
                qk["qctl"][r].copy_(qk["qctl0"][r])
                qk["qslot"][r].copy_(qk["qslot0"][r])
            qk["done"].zero_()
            qk["rdy"].zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if qk is not None:
            _lib.check(self.lib.dpl_dtr_potrf_q(self.args_d.data_ptr(), self.nwg, _lib.stream_ptr()),
                       "dtr_potrf_q (emulation)")
        else:
            _lib.check(self.lib.dpl_dtr_potrf(self.args_d.data_ptr(), self.nwg, _lib.stream_ptr()),
                       "dtr_potrf (emulation)")
        torch.cuda.synchronize()
        span = time.perf_counter() - t0
        r = int(self.info.item())
        if r != 0:
            raise RuntimeError(f"emulated potrf: info {r}")
        return span

    def assemble(self):
        """The factor as one one-process descriptor (lower tiles from their owners)."""
        import torch

        from .. import descriptor as dsc
        N, nt = self.N, self.N // NBT
        L = dsc.TiledMatrix(torch.float64, NBT, NBT, N, N, device=self.ctx.device)
        A0 = dsc.TiledMatrix(torch.float64, NBT, NBT, N, N, device=self.ctx.device)
        for j in range(nt):
            for i in range(j, nt):
                r = self.plan._owner(i, j)
                Ar = self.A[r]
                o = Ar.offset(i, j)
                L.data[L.offset(i, j): L.offset(i, j) + NBT * NBT].copy_(Ar.data[o:o + NBT * NBT])
                A0.data[A0.offset(i, j): A0.offset(i, j) + NBT * NBT].copy_(self.A0[r][o:o + NBT * NBT])
        return L, A0


# ------------------------------------------------------------------------------------ process mode
class _Peers:
    """This rank's receive buffer, W and counters, exported over IPC, and every peer's mapped into this
    process (one process per GPU; ranks sharing a GPU -- the rehearsal -- work the same way)."""

    def __init__(self, ctx, specs):
        import ctypes

        import torch.distributed as dist

        from ..ops import _lib
        lib = _lib.load()
        self.lib = lib
        self.local, self.opened = [], []
        hb = int(lib.dpl_ipc_handle_bytes())
        mine, err = [], None
        # A failure on one rank (allocation, mapping) is agreed through the gathers below, never raised before
        # them: every rank reaches the same collectives and raises together, and close() (collective) runs on
        # every rank because the object is registered before anything can raise.
        _PEERS.append(self)
        for nbytes, cached in specs:
            h = (ctypes.c_char * hb)()
            ptr = ctypes.c_void_p()
            rc = lib.dpl_ipc_alloc(int(nbytes), int(cached), ctypes.byref(ptr), h)
            if rc != 0:
                err = f"rank {ctx.rank}: IPC allocation of {nbytes} bytes failed ({rc})"
                break
            self.local.append(ptr.value)
            mine.append(bytes(h))
        allh = [None] * ctx.world
        dist.all_gather_object(allh, (err, mine))
        errs = [e for e, _ in allh if e]
        if errs:
            raise RuntimeError("distributed DTR: " + "; ".join(errs))
        self.ptrs = []          # [buffer][rank] -> device pointer in this process
        for b in range(len(specs)):
            row = []
            for r in range(ctx.world):
                if r == ctx.rank or err:
                    row.append(self.local[b] if r == ctx.rank else 0)
                    continue
                p = ctypes.c_void_p()
                rc = lib.dpl_xchg_open(ctypes.create_string_buffer(allh[r][1][b], hb), ctypes.byref(p))
                if rc != 0:
                    err = f"rank {ctx.rank}: cannot map rank {r}'s buffer {b} ({rc})"
                    row.append(0)
                    continue
                self.opened.append(p.value)
                row.append(p.value)
            self.ptrs.append(row)
        errs = [None] * ctx.world
        dist.all_gather_object(errs, err)
        errs = [e for e in errs if e]
        if errs:
            raise RuntimeError("distributed DTR: " + "; ".join(errs))

    def close(self):
        import ctypes

        import torch
        import torch.distributed as dist
        if self.local is None:
            return
        torch.cuda.synchronize()
        if dist.is_initialized():
            dist.barrier()
        for p in self.opened:
            self.lib.dpl_xchg_close(ctypes.c_void_p(p))
        if dist.is_initialized():
            dist.barrier()
        for p in self.local:
            self.lib.dpl_xchg_free(ctypes.c_void_p(p))
        self.local, self.opened = None, []


_PEERS = []


def release_all():
    """Unmap and free the distributed DTR's IPC buffers (every rank; collective)."""
    while _PEERS:
        _PEERS.pop().close()


def _at_exit():
    try:
        import torch.distributed as dist
        if _PEERS and dist.is_available() and dist.is_initialized():
            release_all()
    except Exception:   # pragma: no cover - teardown best effort
        pass


import atexit  # noqa: E402
atexit.register(_at_exit)


def supported(ctx, uplo, A) -> bool:
    from ..constants import dplasmaLower
    from ..descriptor import STORAGE_TILE
    import torch
    if not (ctx.is_gpu and ctx.world > 1 and ctx.world <= 8 and not getattr(ctx, "loopback", False)):
        return False
    if uplo != dplasmaLower or A.dtype != torch.float64 or A.mb != NBT or A.nb != NBT:
        return False
    if A.m != A.n or A.m % NBT or A.storage != STORAGE_TILE or A.grid.P * A.grid.Q != ctx.world:
        return False
    return not (A.it0 or A.jt0 or A.grid.kp != 1 or A.grid.kq != 1 or A.grid.ip or A.grid.jq)


_DPLANS = {}


def potrf_dtr_dist_New(ctx, uplo: int, A, info_out=None):
    """The distributed DTR Cholesky of this rank's tiles (one process per GPU, every rank calls it).
    Each run: counters cleared, a barrier (no peer may send into a counter before it is cleared), one
    persistent launch; info all-reduced."""
    import os

    import torch
    import torch.distributed as dist

    from ..ops import _lib
    from ..parallel import comm
    from ..runtime.taskpool import Taskpool
    from ..utils.flops import flops
    if not supported(ctx, uplo, A):
        raise ValueError("distributed DTR: lower, fp64, NB = 512 TILE storage on the context's P x Q grid (<= 8 GPUs)")
    P, Q, me = A.grid.P, A.grid.Q, ctx.rank
    nt = A.nt
    Dd = max(1, int(os.environ.get("DPLASMA_DTR_DEFER", "4")))
    order = os.environ.get("DPLASMA_DTR_LO_ORDER", "column")
    key = (nt, Dd, P, Q, order)
    plan = _DPLANS.get(key)
    if plan is None:
        plan = _DPLANS[key] = DistPlan(nt, Dd, P, Q, lo_order=order)
    lib = _lib.load()
    img = D.ArgsImage(lib)
    PST = img.pstride
    dev = A.device
    hi, hi_off, lo, lo_off = plan.lists({me: list(range(8))})
    sched = os.environ.get("DPLASMA_DTR_SCHED", "queue")
    # receive buffer and W: cached device memory (operands of many update tasks); DPLASMA_DTR_RECV_UNCACHED=1 puts
    # them in uncached memory instead (a diagnostic for peers whose stores a consumer might read stale)
    rc_ = os.environ.get("DPLASMA_DTR_RECV_UNCACHED", "0") != "1"
    specs = [(plan.recv_elems(me) * 8, rc_), (nt * NBT * NBT * 8, rc_), (plan.ncnt * 4, False)]
    qp = None
    if sched == "queue":
        qp = plan.queue()
        nring = D.NCLASS * 8
        specs += [(len(plan.tasks) * 4, False), (2 * nring * PST * 4, False), (len(qp["qinit"][me]) * 4, False)]
    peers = _Peers(ctx, specs)
    recv_p, W_p, cnt_p = peers.ptrs[:3]

    def up(x):
        return torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    tab = plan.tile_table(me, A.offset, (recv_p[me] - A.data.data_ptr()) // 8)
    assert (recv_p[me] - A.data.data_ptr()) % 8 == 0
    tabs = np.full(plan.nranks * nt * nt, -1, dtype=np.int64)
    tabs[me * nt * nt:(me + 1) * nt * nt] = tab
    keep = dict(tasks=up(plan.tasks.view(np.uint8)), reqs=up(plan.reqs), tab=up(tabs), xoff=up(plan.xoff),
                hi=up(hi if len(hi) else np.zeros(1, dtype=np.int32)), lo=up(lo if len(lo) else np.zeros(1, dtype=np.int32)),
                hs=up(plan.hs_off))
    cur = torch.zeros((img.maxr + 8) * PST, dtype=torch.int32, device=dev)
    scur = torch.zeros(plan.nranks * nt * PST, dtype=torch.int32, device=dev)
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    scr = D.PotrfScratch(nt, dev, PST)
    img.set("ld", NBT)
    img.set("nt", nt)
    img.set("nranks", plan.nranks)
    img.set("rank", me)
    img.set("dil", 1)
    img.set("ncnt", plan.ncnt)
    for f in ("tasks", "reqs", "tab", "xoff", "hi", "lo"):
        img.set(f, keep[f].data_ptr())
    img.set("hs_off", keep["hs"].data_ptr())
    img.set("nsteps", nt)
    img.set("scur", scur.data_ptr())
    img.set("cur", cur.data_ptr())
    img.set("hi_off", hi_off)
    img.set("lo_off", lo_off)
    img.set("A", [A.data.data_ptr() if r == me else 0 for r in range(plan.nranks)])
    img.set("recv", recv_p)
    img.set("W", W_p)
    img.set("cnt", cnt_p)
    scr.fill(img)
    img.set("info", info.data_ptr())
    img.set("flags", D.flags_from_env())
    qk = None
    if qp is not None:
        pend_p, qctl_p, qslot_p = peers.ptrs[3:6]
        qctl0 = torch.zeros(2 * nring * PST, dtype=torch.int32)
        qctl0.view(nring, 2, PST)[:, 1, 0] = torch.from_numpy(qp["tinit"][me])
        qk = {"pend0": up(qp["ndeps"]), "qctl0": qctl0.to(dev), "qslot0": up(qp["qinit"][me]),
              "succ_off": up(qp["succ_off"]), "succ": up(qp["succ"]), "ring_of": up(qp["ring_of"]),
              "town": up(qp["town"]), "qbase": up(qp["qbase"]), "done": torch.zeros(1, dtype=torch.int32, device=dev)}
        img.set("ntask", qp["nown"][me])
        img.set("nclass", D.NCLASS)
        for f in ("succ_off", "succ", "ring_of", "town", "qbase", "done"):
            img.set(f, qk[f].data_ptr())
        img.set("pend", pend_p)
        img.set("qctl", qctl_p)
        img.set("qslot", qslot_p)
        keep["q"] = qk
    args_d = torch.empty(img.size, dtype=torch.uint8, device=dev)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    nwg = int(os.environ.get("DPLASMA_DTR_WG", ncu))   # one per CU (see models/potrf_dtr.py)
    nwg = max(64, min(nwg, 2 * ncu))
    cnt_local = torch.empty(0)   # (the counters live in the IPC buffer: cleared by a memset kernel below)
    tp = Taskpool("potrf", ctx)
    tp.flops = flops(A.prec, "potrf", A.n)
    tp.info = info
    state = {"epoch": 0}
    tp._keep = (keep, cur, scur, info, scr, args_d, peers, cnt_local)
    tp.dtr_plan = plan

    def f_run():
        state["epoch"] = state["epoch"] % ((1 << 25) - 1) + 1
        img.set("epoch", state["epoch"])
        args_d.copy_(torch.frombuffer(bytearray(img.buf), dtype=torch.uint8))
        cur.zero_()
        scur.zero_()
        torch.cuda.current_stream().synchronize()
        _lib.check(lib.dpl_memset_sync(cnt_p[me], 0, plan.ncnt * 4), "dtr counters")
        if qk is not None:
            # this rank's pending counts and rings from their templates (peers push into them after the barrier)
            for dst, src in ((pend_p[me], qk["pend0"]), (qctl_p[me], qk["qctl0"]), (qslot_p[me], qk["qslot0"])):
                _lib.check(lib.dpl_memcpy_sync(dst, src.data_ptr(), src.numel() * 4), "dtr queue reset")
            qk["done"].zero_()
            torch.cuda.current_stream().synchronize()
        # every rank's counters are cleared before any rank's kernel can send into them
        comm.barrier_world()
        if qk is not None:
            _lib.check(lib.dpl_dtr_potrf_q(args_d.data_ptr(), nwg, _lib.stream_ptr()), "dtr_potrf_q (distributed)")
            return
        _lib.check(lib.dpl_dtr_potrf(args_d.data_ptr(), nwg, _lib.stream_ptr()), "dtr_potrf (distributed)")

    tp.task("DTR_POTRF", "update", f_run)

    def poison():
        """NaN-fill (0xFF bytes) this rank's receive slots and every W_k it does not compute itself, so a consumer
        that reads a peer's strip or W block before it has arrived gets NaN -- a residual failure -- instead of the
        bit-identical values an earlier factorisation of the same matrix left there (bench.py's engine race).  W_k
        of a diagonal tile this rank owns stays as it is: w_column writes its upper blocks only, the zeros below
        the diagonal come from the allocation."""
        torch.cuda.current_stream().synchronize()
        _lib.check(lib.dpl_memset_sync(recv_p[me], 0xFF, plan.recv_elems(me) * 8), "dtr poison recv")
        blk = NBT * NBT * 8
        k = 0
        while k < nt:
            if A.rank_of(k, k) == me:
                k += 1
                continue
            k1 = k
            while k1 < nt and A.rank_of(k1, k1) != me:
                k1 += 1
            _lib.check(lib.dpl_memset_sync(W_p[me] + k * blk, 0xFF, (k1 - k) * blk), "dtr poison W")
            k = k1
    tp.poison = poison

    def _done():
        v = info.to(torch.int64)
        if dist.get_backend() != "nccl":
            v = v.cpu()
        neg = torch.where(v < 0, v, torch.zeros_like(v))
        dist.all_reduce(neg, op=dist.ReduceOp.MIN)
        if int(neg.item()) < 0:
            raise RuntimeError(f"potrf: distributed device task runtime failure (info {int(neg.item())})")
        pos = torch.where(v > 0, v, torch.full_like(v, 1 << 40))
        dist.all_reduce(pos, op=dist.ReduceOp.MIN)
        r = int(pos.item())
        r = 0 if r == 1 << 40 else r
        if info_out is not None:
            info_out[0] = r
        return r
    tp.on_complete(_done)
    return tp.finish_build()
