"""TileProgram: bulk-synchronous, owner-computes tile programs over P x Q grids.

This is the generic execution model behind every algorithm that does not have
a hand-scheduled stream program (TRSM/TRMM variants, TRTRI, LAUUM, POTRI,
POINV, LU, QR, ...).  It plays the role PaRSEC's PTG plays for the reference
(``src/*.jdf``: task classes with owner-computes placement ``: descA(m,n)`` and
dataflow edges that become MPI messages when they cross ranks), re-designed
for one-process-per-GPU execution with batched kernels:

* An algorithm is built (at ``_New`` time, identically on every rank) as a
  sequence of *stages*.  A stage is a set of independent tile operations
  (GEMM-accumulate, TRSM, POTRF, GETRF, copies, scales, custom tile kernels),
  each writing one output tile; the op runs on the rank owning that tile.
* Reads see the values left by previous stages (stages are the dependency
  frontier -- the analogue of a DAG level).
* For every stage the builder computes, for every rank, which input tiles it
  does not own.  They travel as ONE dataflow exchange per stage
  (``parallel.p2p``: grouped RCCL send/recv with only the peers involved, on a
  communication stream) issued right after the last stage that writes any of
  them -- so it overlaps the stages in between -- and received in place into
  one of ``RING`` pre-allocated receive slabs; the stage then runs ONE batched
  kernel launch per (op kind, operand sources) group -- e.g. all GEMM updates
  of a step in a single MFMA launch.
* On a single rank there is no exchange at all and every operand is read in
  place.
"""
from __future__ import annotations

from collections import defaultdict
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np
import torch

from ..constants import dplasmaNoTrans
from ..ops import tile_ops as ops
from ..ops.batch import GemmBatch, TileBatch
from ..utils import trace
from .taskpool import Taskpool

Key = Tuple[int, int, int]  # (matrix id, m, n)


class _Op:
    __slots__ = ("kind", "out", "ins", "params")

    def __init__(self, kind, out, ins, params):
        self.kind, self.out, self.ins, self.params = kind, out, ins, params


class Stage:
    def __init__(self, prog: "TileProgram", name: str):
        self.prog = prog
        self.name = name
        self.ops: List[_Op] = []

    # -- op constructors; tiles are (M, m, n) with M a TiledMatrix registered on the fly
    def _k(self, t) -> Key:
        M, m, n = t
        return (self.prog.mid(M), m, n)

    def gemm(self, C, terms, alpha=1.0, beta=1.0, mask: int = 0):
        """C = beta*C + alpha * sum_t opA_t(A_t) opB_t(B_t); terms: [(A, opA, B, opB)].
        Terms with different (opA, opB) are allowed (split into launches)."""
        t = [(self._k(a), oa, self._k(b), ob) for (a, oa, b, ob) in terms]
        ins = [x[0] for x in t] + [x[2] for x in t]
        self.ops.append(_Op("gemm", self._k(C), ins, (t, alpha, beta, mask)))
        return self

    def trsm(self, side, uplo, trans, diag, alpha, T, B):
        self.ops.append(_Op("trsm", self._k(B), [self._k(T)], (side, uplo, trans, diag, alpha)))
        return self

    def potrf(self, uplo, A, info, info_base):
        self.ops.append(_Op("potrf", self._k(A), [], (uplo, info, info_base)))
        return self

    def copy(self, src, dst, part=0, trans=dplasmaNoTrans):
        self.ops.append(_Op("copy", self._k(dst), [self._k(src)], (part, trans)))
        return self

    def geadd(self, src, dst, alpha, beta, part=0, trans=dplasmaNoTrans):
        self.ops.append(_Op("geadd", self._k(dst), [self._k(src)], (part, trans, alpha, beta)))
        return self

    def laset(self, dst, part, alpha, beta):
        self.ops.append(_Op("laset", self._k(dst), [], (part, alpha, beta)))
        return self

    def lascal(self, dst, part, alpha):
        self.ops.append(_Op("lascal", self._k(dst), [], (part, alpha)))
        return self

    def tile_fn(self, out, ins, fn: Callable, key=None):
        """Custom tile op: fn(out_view, [in_views]) runs per tile (CPU/GPU tensor views).
        ``key`` groups ops that can share one batched implementation (see tile_batch_fn)."""
        self.ops.append(_Op("fn", self._k(out), [self._k(i) for i in ins], (fn,)))
        return self

    def batch_fn(self, out_tiles, in_tiles, fn: Callable):
        """Custom batched op: fn(resolved) where resolved maps every tile key to (base, off, ld).
        All out tiles must be local to the same rank set as a regular op (owner of out_tiles[0])."""
        outs = [self._k(o) for o in out_tiles]
        ins = [self._k(i) for i in in_tiles]
        self.ops.append(_Op("batch", outs[0], ins, (fn, outs)))
        return self


class TileProgram:
    def __init__(self, ctx, name: str):
        self.ctx = ctx
        self.name = name
        self.mats = []
        self._mid = {}
        self.stages: List[Stage] = []
        self.flops = 0.0
        self._compiled = None

    def mid(self, M) -> int:
        k = id(M)
        if k not in self._mid:
            self._mid[k] = len(self.mats)
            self.mats.append(M)
        return self._mid[k]

    def stage(self, name: str = "") -> Stage:
        s = Stage(self, name or f"S{len(self.stages)}")
        self.stages.append(s)
        return s

    # ------------------------------------------------------------------ compile
    def _owner(self, key: Key) -> int:
        M = self.mats[key[0]]
        return M.rank_of(key[1], key[2])

    def compile(self) -> Taskpool:
        ctx = self.ctx
        me = ctx.rank
        tp = Taskpool(self.name, ctx)
        tp.flops = self.flops
        # loopback rehearsal (parallel.comm.loopback): one rank, every operand edge through the transport
        self._loop = bool(getattr(ctx, "loopback", False))
        distributed = ctx.world > 1 or self._loop
        dtype = self.mats[0].dtype if self.mats else torch.float64
        stages = [st for st in self.stages if st.ops]
        self.transport = None
        layouts: List[Optional[_RecvLayout]] = [None] * len(stages)
        if distributed and stages:
            self.transport = self._plan_transport(stages, layouts, dtype)
        runners = []
        for si, st in enumerate(stages):
            my_ops = [op for op in st.ops if self._owner(op.out) == me]
            runners.append(_StageRunner(self, st, my_ops, layouts[si]))
        tr = self.transport
        prev = None
        for si, runner in enumerate(runners):
            def fn(si=si, runner=runner, last=(si == len(runners) - 1)):
                s = torch.cuda.current_stream(ctx.device) if ctx.is_gpu else None
                if tr is not None:
                    if si == 0:
                        tr.start(s)
                    tr.before(si, s)
                    runner.buf = self._ring[si % len(self._ring)] if self._ring else None
                runner.run()
                if tr is not None:
                    tr.after(si, s)
                    if last:
                        tr.finish(s)
            prev = tp.task(runner.st.name, "update", fn, [prev])
        tp.transport = tr
        return tp.finish_build()

    RING = 3   # receive slabs in flight: a stage's operands may arrive up to RING-1 stages early

    def _plan_transport(self, stages, layouts, dtype):
        """Dataflow exchanges (parallel.p2p): stage s's remote operands travel in one exchange
        issued right after the last stage that writes any of them (and no earlier than stage
        s - RING, whose receive slab it reuses), received in place into the slab."""
        from ..parallel.p2p import Transport, Xfer, first_after
        ctx, me, world = self.ctx, self.ctx.rank, self.ctx.world
        mb = max(M.mb for M in self.mats)
        nb = max(M.nb for M in self.mats)
        nbe = mb * nb
        K = self.RING
        nmat = len(self.mats)
        last_w: Dict[Key, int] = {}
        my_writes_k, my_writes_s = [], []
        kid: Dict[Key, int] = {}

        def kcode(key):
            c = kid.get(key)
            if c is None:
                c = kid[key] = len(kid)
            return c
        plans = []
        for si, st in enumerate(stages):
            needs = defaultdict(list)
            seen = defaultdict(set)
            ready = -1
            for op in st.ops:
                o = self._owner(op.out)
                for k in op.ins:
                    if (self._owner(k) != o or (self._loop and k != op.out)) and k not in seen[o]:
                        seen[o].add(k)
                        needs[o].append(k)
                        ready = max(ready, last_w.get(k, -1))
            for op in st.ops:
                last_w[op.out] = si
                if self._owner(op.out) == me:
                    my_writes_k.append(kcode(op.out))
                    my_writes_s.append(si)
            if any(needs.values()):
                plans.append((si, dict(needs), max(ready, si - K)))
        tr = Transport(ctx, self.name, lambda: [M.data for M in self.mats] + list(self._ring))
        maxrecv = 0
        wk = np.array(my_writes_k, dtype=np.int64)
        ws = np.array(my_writes_s, dtype=np.int64)
        for si, needs, point in plans:
            lay = _RecvLayout(self.mats, needs.get(me, []), mb, nbe, self._owner)
            layouts[si] = lay
            maxrecv = max(maxrecv, lay.nrecv)
            sends = defaultdict(list)
            for d in range(world):
                for key in needs.get(d, []):
                    if self._owner(key) == me and (d != me or self._loop):
                        M = self.mats[key[0]]
                        sends[d].append((key[0], M.offset(key[1], key[2]), M.ld, M.tile_rows(key[1]),
                                         M.tile_cols(key[2]), mb))
            recvs = defaultdict(list)
            for key in needs.get(me, []):
                M = self.mats[key[0]]
                recvs[self._owner(key)].append((nmat + si % K, lay.slot[key], mb, M.tile_rows(key[1]),
                                                M.tile_cols(key[2]), mb))
            x = Xfer(si, dtype, nbe, sends, recvs, label=f"{self.name}:{si}",
                     recv_into=(nmat + si % K, 0))
            guard = None
            if x.send_peers:
                sk = np.array([kcode(key) for d in sends for key in
                               [k for k in needs.get(d, []) if self._owner(k) == me]], dtype=np.int64)
                gx = first_after(wk, ws, sk, np.full(len(sk), point), len(stages))
                gx = gx[gx >= 0]
                guard = int(gx.min()) if len(gx) else None
            tr.add(x, point, si if x.recv_peers else None, guard)
        tr.n_global = len(plans)
        ring = min(K, len(stages))
        self._ring = [torch.empty(max(1, maxrecv) * nbe, dtype=dtype, device=ctx.device) for _ in range(ring)] \
            if maxrecv else []
        return tr

    def execute(self):
        return self.compile().execute(self.ctx)


class _RecvLayout:
    """Where a stage's remote operands sit in its receive slab: by source rank, in need order,
    one mb x nb slot each (ld = mb) -- the layout the exchange receives in place."""

    def __init__(self, mats, mine: List[Key], mb: int, nbe: int, owner):
        self.ld = mb
        by_src = defaultdict(list)
        for key in mine:
            by_src[owner(key)].append(key)
        self.slot: Dict[Key, int] = {}
        pos = 0
        for s in sorted(by_src):
            for key in by_src[s]:
                self.slot[key] = pos * nbe
                pos += 1
        self.nrecv = pos

    def offset(self, mid: int, m: int, n: int) -> int:
        return self.slot[(mid, m, n)]


class _StageRunner:
    """Resolves operand locations and groups the rank's ops into batched launches."""

    def __init__(self, prog: TileProgram, st: Stage, my_ops: List[_Op], plan: Optional["_RecvLayout"]):
        self.prog, self.st, self.plan = prog, st, plan
        self.buf = None  # this stage's receive slab (set by the program before each run)
        self.launches = []
        mats = prog.mats

        def loc(key: Key):
            M = mats[key[0]]
            if plan is None or key not in plan.slot:   # local (the receive plan holds every remote operand)
                return ("L", key[0]), M.offset(key[1], key[2]), M.ld
            return ("R", 0), plan.offset(*key), plan.ld

        def base_of(src):
            return mats[src[1]].data if src[0] == "L" else self.buf

        self._base_of = base_of
        # ---- GEMM: group by (opA, opB, srcA, srcB, C matrix, alpha, beta-class)
        gg: Dict[tuple, GemmBatch] = {}
        for op in my_ops:
            if op.kind != "gemm":
                continue
            terms, alpha, beta, mask = op.params
            C = mats[op.out[0]]
            coff = C.offset(op.out[1], op.out[2])
            rows, cols = C.tile_rows(op.out[1]), C.tile_cols(op.out[2])
            by = defaultdict(list)
            for (ka, oa, kb, ob) in terms:
                sa, aoff, lda = loc(ka)
                sb, boff, ldb = loc(kb)
                A = mats[ka[0]]
                kext = A.tile_cols(ka[2]) if oa == dplasmaNoTrans else A.tile_rows(ka[1])
                by[(oa, ob, sa, sb, lda, ldb)].append((aoff, boff, kext))
            first = True
            for gk, kps in by.items():
                b_eff = beta if first else 1.0
                key = gk + (op.out[0], alpha, b_eff, first)
                first = False
                gb = gg.get(key)
                if gb is None:
                    gb = gg[key] = GemmBatch()
                gb.add(coff, rows, cols, kps, mask)
            if not terms and beta != 1.0:
                # pure scaling
                self._scal(op.out, beta)
        # a C tile may appear in several groups: groups sharing a C tile must run in order
        # (first group applies beta); launch order = insertion order keeps that.
        # groups holding an op's FIRST term (they apply beta) launch before the rest
        for key, gb in sorted(gg.items(), key=lambda kv: not kv[0][-1]):
            (oa, ob, sa, sb, lda, ldb, cm, alpha, b_eff, _first) = key
            gb.finalize()
            self.launches.append(("gemm", (oa, ob, sa, sb, lda, ldb, cm, alpha, b_eff, gb)))
        # ---- TRSM: group by (params, srcT, B matrix)
        tg: Dict[tuple, TileBatch] = {}
        for op in my_ops:
            if op.kind != "trsm":
                continue
            side, uplo, trans, diag, alpha = op.params
            st_, toff, ldt = loc(op.ins[0])
            B = mats[op.out[0]]
            key = (side, uplo, trans, diag, alpha, st_, ldt, op.out[0])
            tb = tg.setdefault(key, TileBatch())
            tb.add(toff, B.tile_rows(op.out[1]), B.tile_cols(op.out[2]), b_off=B.offset(op.out[1], op.out[2]))
        for key, tb in tg.items():
            tb.finalize()
            self.launches.append(("trsm", key + (tb,)))
        # ---- others: one launch per op (potrf) or grouped maps
        for op in my_ops:
            if op.kind == "potrf":
                uplo, info, info_base = op.params
                A = mats[op.out[0]]
                self.launches.append(("potrf", (uplo, op.out[0], A.offset(op.out[1], op.out[2]),
                                                A.tile_rows(op.out[1]), info, info_base)))
        mg: Dict[tuple, TileBatch] = {}
        for op in my_ops:
            if op.kind in ("copy", "geadd"):
                D = mats[op.out[0]]
                s_, soff, lds_ = loc(op.ins[0])
                if op.kind == "copy":
                    part, trans = op.params
                    key = ("copy", part, trans, s_, lds_, op.out[0], 1.0, 0.0)
                else:
                    part, trans, alpha, beta = op.params
                    key = ("geadd", part, trans, s_, lds_, op.out[0], alpha, beta)
                tb = mg.setdefault(key, TileBatch())
                tb.add(soff, D.tile_rows(op.out[1]), D.tile_cols(op.out[2]), gi=op.out[1] * D.mb,
                       gj=op.out[2] * D.nb, b_off=D.offset(op.out[1], op.out[2]))
            elif op.kind in ("laset", "lascal"):
                D = mats[op.out[0]]
                key = (op.kind,) + tuple(op.params) + (op.out[0],)
                tb = mg.setdefault(key, TileBatch())
                tb.add(D.offset(op.out[1], op.out[2]), D.tile_rows(op.out[1]), D.tile_cols(op.out[2]),
                       gi=op.out[1] * D.mb, gj=op.out[2] * D.nb)
        for key, tb in mg.items():
            tb.finalize()
            self.launches.append(("map", key + (tb,)))
        for op in my_ops:
            if op.kind == "fn":
                self.launches.append(("fn", (op, [loc(k) for k in op.ins])))
            elif op.kind == "batch":
                fn, outs = op.params
                res = {}
                for k in list(op.ins) + list(outs):
                    res[k] = loc(k)
                self.launches.append(("batch", (fn, res)))

    def _scal(self, out, beta):
        M = self.prog.mats[out[0]]
        tb = TileBatch().add(M.offset(out[1], out[2]), M.tile_rows(out[1]), M.tile_cols(out[2]),
                             gi=out[1] * M.mb, gj=out[2] * M.nb).finalize()
        self.launches.append(("map", ("lascal", 0, beta, out[0], tb)))

    def run(self):
        with trace.span(self.prog.ctx, f"{self.prog.name}:{self.st.name}", "stage",
                        args={"launches": len(self.launches), "exchange": self.plan is not None}):
            self._run()

    def _run(self):
        mats = self.prog.mats
        B = self._base_of
        for kind, p in self.launches:
            if kind == "gemm":
                oa, ob, sa, sb, lda, ldb, cm, alpha, b_eff, gb = p
                C = mats[cm]
                ops.gemm(oa, ob, alpha, B(sa), lda, B(sb), ldb, b_eff, C.data, C.ld, gb)
            elif kind == "trsm":
                side, uplo, trans, diag, alpha, st_, ldt, bm, tb = p
                Bm = mats[bm]
                ops.trsm(side, uplo, trans, diag, alpha, B(st_), ldt, Bm.data, Bm.ld, tb)
            elif kind == "potrf":
                uplo, am, off, n, info, info_base = p
                A = mats[am]
                ops.potrf_tile(uplo, A.data, off, n, A.ld, info, info_base)
            elif kind == "map":
                k0 = p[0]
                if k0 in ("copy", "geadd"):
                    _, part, trans, s_, lds_, dm, alpha, beta, tb = p
                    D = mats[dm]
                    ops.geadd(part, trans, alpha, B(s_), lds_, beta, D.data, D.ld, tb, copy=(k0 == "copy"))
                elif k0 == "laset":
                    _, part, alpha, beta, dm, tb = p
                    D = mats[dm]
                    ops.laset(part, alpha, beta, D.data, D.ld, tb)
                elif k0 == "lascal":
                    _, part, alpha, dm, tb = p
                    D = mats[dm]
                    ops.lascal(part, alpha, D.data, D.ld, tb)
            elif kind == "fn":
                op, locs = p
                M = mats[op.out[0]]
                outv = M.tile(op.out[1], op.out[2])
                ins = []
                for (src, off, ld), k in zip(locs, op.ins):
                    Mi = mats[k[0]]
                    r, c = Mi.tile_rows(k[1]), Mi.tile_cols(k[2])
                    ins.append(torch.as_strided(B(src), (r, c), (1, ld), off))
                op.params[0](outv, ins)
            elif kind == "batch":
                fn, res = p
                fn({k: (B(v[0]), v[1], v[2]) for k, v in res.items()})
