"""Tile-task DAGs executed as level-synchronous batched launches.

This is dplasma_amd's counterpart of the reference's two task-graph front
ends -- the PTG/JDF algorithms (e.g. ``src/zgeqrf.jdf``, ``src/zgeqrf_param.jdf``,
``src/zgetrf_incpiv.jdf``) and the DTD insert-task interface
(``parsec_dtd_insert_task`` as used by ``src/dtd_wrappers/``) -- redesigned for
MI355X:

* An algorithm inserts tile tasks in *program order* (DTD semantics), each
  naming the tiles it reads and writes.  Insertion is vectorised: one call adds
  a whole numpy array of tasks of one kind.
* ``compile()`` computes every task's dependency *level* in native code
  (``csrc/runtime/dag.cpp``: RAW/WAR/WAW hazards per tile).  All tasks of one
  kind in one level are independent, so they become ONE batched kernel launch
  -- thousands of tile updates per launch instead of one tiny launch per task,
  which is what it takes to fill 256 CUs.
* Distributed (one process per GPU): a task executes on the home rank of its
  designated tile (owner-computes, like the JDF's ``: descA(m, n)`` affinity).
  Other tiles it touches are fetched into a per-rank slot arena (cached per
  tile version, so a panel's V/T tiles are fetched once per rank, not once per
  update) straight from the rank holding that version (its home, or the remote
  executor that produced it), and tiles it modifies are written back to their
  home.  Transport is dataflow (``parallel.p2p``): each edge is issued right
  after the level that makes it final, as grouped RCCL send/recv with only the
  peers involved, on a communication stream, and the compute stream waits only
  before the first level that reads it -- the PTG remote dependencies of
  ``src/zgeqrf.jdf:84-121`` without a runtime message engine.

Items carry absolute device addresses (``DAG_ITEM``, 96 bytes: six operand
slots, layout of ``QrItem`` in ``csrc/kernels/qr.hip``) so one launch can mix tiles living in
descriptor storage and in the slot arena.  All items are built and uploaded
once at compile time ("ENQ" phase, excluded from timing as in
``tests/common.h:252-277``).
"""
from __future__ import annotations

import os
from collections import defaultdict
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from ..constants import STORAGE_TILE
from ..utils import trace
from .taskpool import Taskpool

DAG_ITEM = np.dtype([("p0", "<u8"), ("p1", "<u8"), ("p2", "<u8"), ("p3", "<u8"),
                     ("ld0", "<i4"), ("ld1", "<i4"), ("ld2", "<i4"), ("ld3", "<i4"),
                     ("m", "<i4"), ("n", "<i4"), ("k", "<i4"), ("pad", "<i4"),
                     ("p4", "<u8"), ("p5", "<u8"),
                     ("ld4", "<i4"), ("ld5", "<i4"), ("aux0", "<i4"), ("aux1", "<i4")])
assert DAG_ITEM.itemsize == 96

R, W, RW = 1, 2, 3

MULTISTREAM = True  # single-GPU DAGs: critical-path stream + bulk stream
# DPLASMA_PTG_TO_DTD=1: every tile DAG is re-executed through the DTD front end (TileDAG._ptg_to_dtd)
PTG_TO_DTD = [os.environ.get("DPLASMA_PTG_TO_DTD", "0") == "1"]
CRIT_SLACK = 0      # tasks with at most this much slack (levels) go to the critical stream

_MID_SHIFT, _M_SHIFT = 44, 22
_MASK22 = (1 << 22) - 1


def _root(M):
    while getattr(M, "_parent", None) is not None:
        M = M._parent
    return M


@dataclass
class Kind:
    """A tile-kernel family usable in a DAG.

    roles: tuple of (role name, access mode, item pointer slot 0..5)
    exec_role: index of the role whose home rank executes the task
    gpu(items_dev_ptr, nitems, stream_ptr, emax): one batched launch; emax = max (m, n, k) over the items
    cpu(refs, ext): reference execution of one task; refs[r] = (tensor, offset, ld)
    """
    name: str
    roles: Tuple[Tuple[str, int, int], ...]
    exec_role: int
    gpu: Callable
    cpu: Callable
    flops: Optional[Callable] = None  # ext (n, 3) int array -> total flops
    prio: int = 0                     # launch order within a level (lower first)
    # DTD-style task class: body(*tile_views, *pyargs) runs once per task (on the
    # level's stream) instead of one batched launch; gpu/cpu are then unused
    body: Optional[Callable] = None


def _lib_rt():
    try:
        from ..lib import _dplasma_rt as rt  # type: ignore
        return rt
    except Exception:
        return None


def _levels_py(ops, modes):
    st = {}
    out = np.zeros(len(ops), dtype=np.int32)
    for t in range(len(ops)):
        L = 0
        for k, md in zip(ops[t], modes[t]):
            if not md or k not in st:
                continue
            lw, mr = st[k]
            if lw >= L:
                L = lw + 1
            if (md & 2) and mr >= L:
                L = mr + 1
        out[t] = L
        for k, md in zip(ops[t], modes[t]):
            if not md:
                continue
            lw, mr = st.get(k, (-1, -1))
            st[k] = (L, -1) if md & 2 else (lw, max(mr, L))
    return out


def _versions_py(ops, modes):
    ver = defaultdict(int)
    out = np.full(ops.shape, -1, dtype=np.int32)
    for t in range(len(ops)):
        for r in range(ops.shape[1]):
            if modes[t, r]:
                out[t, r] = ver[ops[t, r]]
        for r in range(ops.shape[1]):
            if modes[t, r] & 2:
                ver[ops[t, r]] += 1
    return out


# Reference task costs (JDF ``SIMCOST``): zgeqrf.jdf:105,207,323,454 and zgeqrf_param.jdf:69,147,
# 213,313 (TT kernels cost 2 / 6 instead of the TS 6 / 12).  Other kinds cost 1.
REFERENCE_SIMCOST = {"geqrt": 4, "unmqr": 6, "tsqrt": 6, "ttqrt": 2, "tsmqr": 12, "ttmqr": 6}


def _kernel_of(kind_name: str) -> str:
    """Kernel family of a kind name: "qr0000_tsmqr_h_3_32" -> "tsmqr", "incpiv_getrf_d" -> "getrf"."""
    parts = kind_name.split("_")
    return parts[1] if len(parts) > 1 else kind_name


def simulation_date(ops: np.ndarray, modes: np.ndarray, kid: np.ndarray, kind_names: Sequence[str],
                    cost=None) -> float:
    """Critical-path length of a tile DAG with per-kind task costs: the analogue of PaRSEC's
    simulation date (``parsec_getsimulationdate``, printed by ``tests/testing_zgeqrf_systolic.c:139-150``,
    ``testing_zgelqf.c:97-99``).  A task starts when the last writer of every tile it touches has
    finished (dataflow: RAW and in-place RW chains; reads do not order later writes, as PTG data
    versions do not) and ends ``cost`` later; the date is the latest end.  ``cost``: dict kernel
    family -> cost (default ``REFERENCE_SIMCOST``) or callable(kind name) -> cost."""
    table = REFERENCE_SIMCOST if cost is None else cost
    if callable(table):
        kc = [float(table(n)) for n in kind_names]
    else:
        kc = [float(table.get(_kernel_of(n), 1.0)) for n in kind_names]
    done: Dict[int, float] = {}
    end = 0.0
    for t in range(len(ops)):
        start = 0.0
        for k, md in zip(ops[t], modes[t]):
            if md:
                d = done.get(int(k))
                if d is not None and d > start:
                    start = d
        fin = start + kc[int(kid[t])]
        for k, md in zip(ops[t], modes[t]):
            if md & W:
                done[int(k)] = fin
        if fin > end:
            end = fin
    return end


class TileDAG:
    """Program-order tile task graph (see module docstring)."""

    def __init__(self, ctx, name: str):
        self.ctx = ctx
        self.name = name
        self.mats: List = []        # root descriptors, index = matrix id
        self._mid: Dict[int, int] = {}
        self.kinds: List[Kind] = []
        self._kid: Dict[str, int] = {}
        self._chunks = []           # (kind id, ops (n, R) int64, ext (n, 3) int32)
        self.flops = 0.0
        self.info = None
        self.no_dtd = False         # the DTD engine's own windows (never re-routed through DTD)
        self._has_prio = False      # some task carries a non-zero priority (add(prio=...))
        self._subs = {}             # chunk index -> (n, R, 2) (row, col) origin of each operand in its tile

    # ------------------------------------------------------------ registration
    def mat(self, M) -> int:
        """Register a descriptor (or a view of one); returns the root's matrix id."""
        Rt = _root(M)
        k = id(Rt)
        if k not in self._mid:
            self._mid[k] = len(self.mats)
            self.mats.append(Rt)
        return self._mid[k]

    def keys(self, M, m, n) -> np.ndarray:
        """Tile keys of view tiles (m, n) of M (scalars or arrays)."""
        mid = self.mat(M)
        gm = np.asarray(m, dtype=np.int64) + M.it0
        gn = np.asarray(n, dtype=np.int64) + M.jt0
        return (np.int64(mid) << _MID_SHIFT) | (gm << _M_SHIFT) | gn

    def kind(self, K: Kind) -> int:
        if K.name not in self._kid:
            self._kid[K.name] = len(self.kinds)
            self.kinds.append(K)
        return self._kid[K.name]

    def add(self, K: Kind, ops, ext, pyargs=None, prio=None, sub=None):
        """Append tasks of kind K in program order.

        ops: (n, len(K.roles)) tile keys (-1 for an unused optional role); ext: (n, 3) ints;
        pyargs: optional per-task tuples of Python values passed to a ``body`` kind; prio: optional
        per-task priorities (the DTD ``priority`` argument: higher first among the ready tasks of a
        level, and on the high-priority stream when positive); sub: optional (n, R, 2) (row, col)
        origins of the operands inside their tiles -- a task on a sub-block of its tiles (the
        recursive incarnations); dependencies stay per tile."""
        ops = np.atleast_2d(np.asarray(ops, dtype=np.int64))
        ext = np.atleast_2d(np.asarray(ext, dtype=np.int32))
        if ops.size == 0:
            return
        if ops.shape[1] != len(K.roles) or ext.shape != (ops.shape[0], 3):
            raise ValueError(f"{K.name}: bad task array shapes {ops.shape} {ext.shape}")
        if pyargs is not None and len(pyargs) != len(ops):
            raise ValueError("one pyargs tuple per task")
        if prio is not None:
            prio = np.broadcast_to(np.asarray(prio, dtype=np.int64), (len(ops),)).copy()
            if prio.any():
                self._has_prio = True
        kid = self.kind(K)
        if sub is not None:
            sub = np.broadcast_to(np.asarray(sub, dtype=np.int64), (ops.shape[0], ops.shape[1], 2)).copy()
            if sub.any():
                self._subs[len(self._chunks)] = sub
        self._chunks.append((kid, ops, ext, list(pyargs) if pyargs is not None else None, prio))
        if K.flops is not None:
            self.flops += float(K.flops(ext))

    # ------------------------------------------------------------ geometry helpers
    def _tile_shape(self, key: int):
        if key < 0:
            return (0, 0)
        M = self.mats[key >> _MID_SHIFT]
        gm, gn = (key >> _M_SHIFT) & _MASK22, key & _MASK22
        return (min(M.mb, M.lm - gm * M.mb), min(M.nb, M.ln - gn * M.nb))

    def _home(self, keys: np.ndarray) -> np.ndarray:
        mid = keys >> _MID_SHIFT
        gm = (keys >> _M_SHIFT) & _MASK22
        gn = keys & _MASK22
        out = np.zeros(keys.shape, dtype=np.int64)
        for i, M in enumerate(self.mats):
            sel = mid == i
            if not sel.any():
                continue
            g = M.grid
            pr = (gm[sel] // g.kp + g.ip) % g.P
            pc = (gn[sel] // g.kq + g.jq) % g.Q
            out[sel] = pr * g.Q + pc
        return out

    def _local_offsets(self, keys: np.ndarray) -> np.ndarray:
        """Element offsets of home-local tiles in their root descriptor storage."""
        mid = keys >> _MID_SHIFT
        gm = (keys >> _M_SHIFT) & _MASK22
        gn = keys & _MASK22
        out = np.zeros(keys.shape, dtype=np.int64)
        for i, M in enumerate(self.mats):
            sel = mid == i
            if not sel.any():
                continue
            lrow = np.full(M.lmt, -1, dtype=np.int64)
            lcol = np.full(M.lnt, -1, dtype=np.int64)
            for t, k in M.lrow.items():
                lrow[t] = k
            for t, k in M.lcol.items():
                lcol[t] = k
            il, jl = lrow[gm[sel]], lcol[gn[sel]]
            if (il < 0).any() or (jl < 0).any():
                raise RuntimeError("tile is not local to this rank")
            if M.storage == STORAGE_TILE:
                out[sel] = (jl * M.llmt + il) * M.mb * M.nb
            else:
                out[sel] = il * M.mb + jl * M.nb * M.ld
        return out

    # ------------------------------------------------------------ compile
    def _ptg_to_dtd(self) -> Optional[Taskpool]:
        """Re-execute this task graph through the DTD front end (the reference's ``--mca mca_pins
        ptg_to_dtd`` test mode, tests/Testings.cmake:7,11-12,33-36): every task is inserted in program
        order with its tiles' access modes and the executing role as AFFINITY, and the dependencies
        are rediscovered by the DTD engine.  None when a task cannot be expressed (Python-body kinds
        or optional roles left empty): the graph then runs as built."""
        from . import dtd
        if self._subs or any(self.kinds[k].body is not None or (o < 0).any() for k, o, _, _, _ in self._chunks):
            return None
        dt = dtd.DTDTaskpool(self.ctx, self.name + "[ptg_to_dtd]", window=0)
        mask = (1 << 22) - 1
        for k, o, e, _, pr in self._chunks:
            K = self.kinds[k]
            tc = dt.task_class(K.name, kind=K)
            for t in range(len(o)):
                args = []
                for r, key in enumerate(o[t]):
                    key = int(key)
                    ref = dtd.tile_of(self.mats[key >> _MID_SHIFT], (key >> _M_SHIFT) & mask, key & mask)
                    args.append((ref, K.roles[r][1] | (dtd.AFFINITY if r == K.exec_role else 0)))
                dt.insert_task(tc, *args, tuple(int(x) for x in e[t]),
                               priority=int(pr[t]) if pr is not None else 0)
        self._chunks = []
        dt.flops = self.flops
        tp = dt.compile()
        tp.name = self.name
        tp.ptg_to_dtd = True
        return tp

    def compile(self) -> Taskpool:
        ctx = self.ctx
        me, world = ctx.rank, ctx.world
        # loopback rehearsal (parallel.comm.loopback, one rank): every tile access is planned as a remote
        # one -- operands fetched from their home (myself) into the slot arena, written tiles written
        # back -- so the dataflow transport's RCCL path runs with self as the peer
        loop = bool(getattr(ctx, "loopback", False))
        dist_plan = world > 1 or loop
        if PTG_TO_DTD[0] and not self.no_dtd and self._chunks:
            tp = self._ptg_to_dtd()
            if tp is not None:
                return tp
        tp = Taskpool(self.name, ctx)
        tp.flops = self.flops
        if not self._chunks:
            return tp.finish_build()
        nR = max(len(self.kinds[c[0]].roles) for c in self._chunks)
        ntask = sum(len(c[1]) for c in self._chunks)
        ops = np.full((ntask, nR), -1, dtype=np.int64)
        modes = np.zeros((ntask, nR), dtype=np.uint8)
        kid = np.zeros(ntask, dtype=np.int32)
        ext = np.zeros((ntask, 3), dtype=np.int32)
        pyargs_all = None
        tprio = np.zeros(ntask, dtype=np.int64)
        sub_all = np.zeros((ntask, nR, 2), dtype=np.int64) if self._subs else None
        p = 0
        for ci, (k, o, e, pa, pr) in enumerate(self._chunks):
            n = len(o)
            K = self.kinds[k]
            ops[p:p + n, :o.shape[1]] = o
            if ci in self._subs:
                sub_all[p:p + n, :o.shape[1]] = self._subs[ci]
            for r, (_, md, _) in enumerate(K.roles):
                modes[p:p + n, r] = np.where(o[:, r] >= 0, md, 0)
            kid[p:p + n] = k
            ext[p:p + n] = e
            if pr is not None:
                tprio[p:p + n] = pr
            if pa is not None:
                if pyargs_all is None:
                    pyargs_all = [()] * ntask
                pyargs_all[p:p + n] = pa
            p += n
        self._chunks = []
        self._subs = {}
        names = [K.name for K in self.kinds]
        tp.simulation_date = lambda cost=None: simulation_date(ops, modes, kid, names, cost)
        rt = _lib_rt()
        # single process on a GPU: dataflow over two streams (critical path / bulk)
        multistream = world == 1 and not loop and ctx.device.type == "cuda" and rt is not None and MULTISTREAM
        crit = None
        if multistream:
            level, blevel, esrc, edst = rt.dag_schedule(ops, modes)
            depth = level.astype(np.int64) + blevel
            crit = (depth.max() - depth) <= CRIT_SLACK
        else:
            level = rt.dag_levels(ops, modes) if rt is not None else _levels_py(ops, modes)
        nlev = int(level.max()) + 1
        from . import capped
        if capped.wanted(ctx, self.mats):
            # host-resident operands (or an explicit arena cap): bounded device tile arena, LRU
            return capped.compile_capped(self, tp, ops, modes, kid, ext, pyargs_all, level, DAG_ITEM, sub_all)
        dot = getattr(ctx, "dot_file", None)
        if dot and me == 0:
            self._write_dot(dot, ops, modes, kid, level)
        # executor rank per task
        exec_key = ops[np.arange(ntask), np.array([self.kinds[k].exec_role for k in range(len(self.kinds))])[kid]]
        exe = self._home(exec_key) if world > 1 else np.zeros(ntask, dtype=np.int64)

        # ---------------- remote-tile plan (identical on every rank)
        # rows (src, dst, key, version, need level, issue point, phase): fetches of a tile version
        # into the executor's slot arena, straight from the rank holding it (its home, or the
        # remote executor that produced it), and write-backs of remotely written tiles to their home
        xrows = None
        slot_of: Dict[int, int] = {}
        if dist_plan:
            used = modes > 0
            t_idx, r_idx = np.nonzero(used)
            akeys = ops[t_idx, r_idx]
            home = self._home(akeys)
            aexe = exe[t_idx]
            alev = level[t_idx].astype(np.int64)
            awr = (modes[t_idx, r_idx] & 2) > 0
            rem = (home != aexe) | loop
            self._local_access = (akeys[aexe == me], alev[aexe == me], awr[aexe == me])
            if rem.any():
                ver = rt.dag_versions(ops, modes) if rt is not None else _versions_py(ops, modes)
                aver = ver[t_idx, r_idx].astype(np.int64)
                # producer (level, executor) of every written version: version v+1 comes from the
                # task that wrote while seeing version v
                wk, wv, wl, we = akeys[awr], aver[awr], alev[awr], aexe[awr]
                t_r, k_r, h_r, e_r = t_idx[rem], akeys[rem], home[rem], aexe[rem]
                v_r, w_r, l_r = aver[rem], awr[rem], alev[rem]
                order = np.lexsort((l_r, k_r, e_r))
                t_r, k_r, h_r, e_r, v_r, w_r, l_r = (x[order] for x in (t_r, k_r, h_r, e_r, v_r, w_r, l_r))
                first = np.ones(len(k_r), dtype=bool)
                first[1:] = (k_r[1:] != k_r[:-1]) | (e_r[1:] != e_r[:-1])
                have = np.empty(len(k_r), dtype=np.int64)
                have[1:] = v_r[:-1] + w_r[:-1]
                need = first | (v_r != np.where(first, -1, have))
                prev_l = np.full(len(k_r), -1, dtype=np.int64)
                prev_l[1:] = np.where(first[1:], -1, l_r[:-1])
                fi = np.nonzero(need)[0]
                fk, fv, fl = k_r[fi], v_r[fi], l_r[fi]
                # producer of version fv (fv == 0: the initial data at home, available at the start)
                prod_l = np.full(len(fi), -1, dtype=np.int64)
                src = h_r[fi].copy()
                if len(wk) and (fv > 0).any():
                    uk = np.unique(np.concatenate([wk, fk]))
                    VS = np.int64(int(max(wv.max(), fv.max())) + 2)
                    code_w = np.searchsorted(uk, wk).astype(np.int64) * VS + wv
                    ow = np.argsort(code_w)
                    code_w = code_w[ow]
                    sel = fv > 0
                    code_q = np.searchsorted(uk, fk[sel]).astype(np.int64) * VS + (fv[sel] - 1)
                    pos = np.searchsorted(code_w, code_q)
                    pos = np.minimum(pos, len(code_w) - 1)
                    okp = code_w[pos] == code_q
                    if not okp.all():
                        raise RuntimeError(f"{self.name}: producer of a fetched tile version not found")
                    prod_l[sel] = wl[ow][pos]
                    src[sel] = we[ow][pos]
                point = np.maximum(prod_l, prev_l[fi])
                dst = e_r[fi]
                # the producer itself is the executor: its slot already holds it (an initial fetch from
                # home always moves: on a real grid home != executor; loopback fetches from itself)
                direct = (src != dst) | (prod_l < 0)
                f_rows = np.stack([src, dst, fk, fl, point, np.zeros(len(fi), np.int64)], 1)[direct]
                wi = np.nonzero(w_r)[0]
                w_rows = np.stack([e_r[wi], h_r[wi], k_r[wi], l_r[wi], l_r[wi], np.ones(len(wi), np.int64)], 1)
                xrows = np.concatenate([f_rows, w_rows]) if len(w_rows) else f_rows
                mine = np.unique(k_r[e_r == me])
                cnt = defaultdict(int)
                for k in mine.tolist():
                    dt = self.mats[k >> _MID_SHIFT].dtype
                    slot_of[k] = cnt[dt]
                    cnt[dt] += 1
        # slot arenas: one per dtype (IPIV-like integer descriptors get their own),
        # one slot per remote tile this rank touches
        dtypes = sorted({M.dtype for M in self.mats}, key=str)
        nbe_of = {dt: max(M.mb * M.nb for M in self.mats if M.dtype == dt) for dt in dtypes}
        nslots = defaultdict(int)
        for k, s_ in slot_of.items():
            dt = self.mats[k >> _MID_SHIFT].dtype
            nslots[dt] = max(nslots[dt], s_ + 1)
        device = ctx.device
        self.arenas = {dt: torch.zeros(nslots[dt] * nbe_of[dt], dtype=dt, device=device) for dt in dtypes
                       if nslots[dt]}
        arena_base = {}
        bases = [M.data for M in self.mats]
        for dt, ar in self.arenas.items():
            arena_base[dt] = len(bases)
            bases.append(ar)
        esz = np.array([b.element_size() for b in bases] + [0], dtype=np.uint64)
        mat_dt = [M.dtype for M in self.mats]
        dtype = self.mats[0].dtype

        def resolve(keys, home=False):
            """keys (n,) -> (base index, element offset, ld) arrays for this rank (home: the tiles' own
            storage -- the loopback transport's home side)."""
            keys = np.asarray(keys, dtype=np.int64)
            mid = (keys >> _MID_SHIFT).astype(np.int64)
            bidx = mid.copy()
            off = np.zeros(len(keys), dtype=np.int64)
            ld = np.zeros(len(keys), dtype=np.int32)
            if home:
                loc = np.ones(len(keys), dtype=bool)
            elif loop:
                loc = np.zeros(len(keys), dtype=bool)   # every operand in the slot arena
            else:
                loc = (self._home(keys) == me) if world > 1 else np.ones(len(keys), dtype=bool)
            if loc.any():
                off[loc] = self._local_offsets(keys[loc])
                ld[loc] = np.array([self.mats[i].ld for i in range(len(self.mats))], dtype=np.int32)[mid[loc]]
            if (~loc).any():
                rk = keys[~loc]
                dts = [mat_dt[int(k >> _MID_SHIFT)] for k in rk]
                off[~loc] = np.array([slot_of[int(k)] * nbe_of[dt] for k, dt in zip(rk, dts)], dtype=np.int64)
                bidx[~loc] = np.array([arena_base[dt] for dt in dts], dtype=np.int64)
                ld[~loc] = np.array([self.mats[i].mb for i in range(len(self.mats))], dtype=np.int32)[mid[~loc]]
            return bidx, off, ld

        # ---------------- my launches, grouped by (level, critical first, task priority (higher first),
        # kind prio, kind)
        mine_t = np.nonzero(exe == me)[0] if world > 1 else np.arange(ntask)
        prio = np.array([self.kinds[k].prio for k in range(len(self.kinds))])[kid[mine_t]]
        cflag = (~crit[mine_t]).astype(np.int64) if crit is not None else np.zeros(len(mine_t), dtype=np.int64)
        eff = tprio[mine_t].copy()
        if self._has_prio and len(mine_t):
            # a batched kind stays ONE launch per level: its tasks share their highest priority;
            # Python-body kinds (one call per task) order task by task
            batched = np.array([self.kinds[k].body is None for k in range(len(self.kinds))])[kid[mine_t]]
            if batched.any():
                gk = (level[mine_t].astype(np.int64) * 2 + cflag) * (len(self.kinds) + 1) + kid[mine_t]
                gmax = {}
                for g_, v in zip(gk[batched].tolist(), eff[batched].tolist()):
                    if v > gmax.get(g_, -(1 << 62)):
                        gmax[g_] = v
                eff[batched] = np.array([gmax[g_] for g_ in gk[batched].tolist()], dtype=np.int64)
        order = np.lexsort((mine_t, kid[mine_t], prio, -eff, cflag, level[mine_t]))
        mine_t = mine_t[order]
        groups = []  # execution order: dict(K, start, n, cpu_refs, ext, emax, level, stream)
        all_items = []
        nitems_total = 0
        if len(mine_t):
            lv, kk, tp_ = level[mine_t], kid[mine_t], eff[order]
            cf = cflag[order]
            brk = np.nonzero((lv[1:] != lv[:-1]) | (kk[1:] != kk[:-1]) | (cf[1:] != cf[:-1]) |
                             (tp_[1:] != tp_[:-1]))[0] + 1
            starts = np.concatenate([[0], brk])
            ends = np.concatenate([brk, [len(mine_t)]])
            items = np.zeros(len(mine_t), dtype=DAG_ITEM)
            ptr_arr = np.array([b.data_ptr() for b in bases] + [0], dtype=np.uint64)
            refs_all = []
            for r in range(nR):
                keys = ops[mine_t, r]
                ok = keys >= 0
                b = np.full(len(keys), -1, dtype=np.int64)
                o = np.zeros(len(keys), dtype=np.int64)
                l = np.zeros(len(keys), dtype=np.int32)
                if ok.any():
                    b[ok], o[ok], l[ok] = resolve(keys[ok])
                    if sub_all is not None:   # sub-block operands: origin (row, col) inside the tile
                        o[ok] += sub_all[mine_t, r, 0][ok] + sub_all[mine_t, r, 1][ok] * l[ok].astype(np.int64)
                refs_all.append((b, o, l))
            gid_of_task = np.zeros(ntask, dtype=np.int64)
            for g, (s, e) in enumerate(zip(starts, ends)):
                K = self.kinds[int(kk[s])]
                seg = items[s:e]
                for r, (_, _, slot) in enumerate(K.roles):
                    b, o, l = (x[s:e] for x in refs_all[r])
                    addr = ptr_arr[b] + o.astype(np.uint64) * esz[b]  # b == -1 -> trailing 0 entries
                    addr[b < 0] = 0
                    seg[f"p{slot}"] = addr
                    seg[f"ld{slot}"] = l
                seg["m"], seg["n"], seg["k"] = ext[mine_t[s:e], 0], ext[mine_t[s:e], 1], ext[mine_t[s:e], 2]
                cpu_refs = None
                if device.type != "cuda" or K.body is not None:
                    cpu_refs = [[(bases[int(refs_all[r][0][i])] if refs_all[r][0][i] >= 0 else None,
                                  int(refs_all[r][1][i]), int(refs_all[r][2][i])) for r in range(len(K.roles))]
                                for i in range(s, e)]
                ex = ext[mine_t[s:e]]
                gid_of_task[mine_t[s:e]] = g
                pyargs = [pyargs_all[int(t)] for t in mine_t[s:e]] if pyargs_all is not None else None
                shapes = None
                if K.body is not None:
                    shapes = [[self._tile_shape(int(ops[t, r])) for r in range(len(K.roles))] for t in mine_t[s:e]]
                groups.append(dict(K=K, start=int(s), n=int(e - s), cpu_refs=cpu_refs, ext=ex, pyargs=pyargs,
                                   shapes=shapes,
                                   emax=tuple(int(x) for x in ex.max(0)), level=int(lv[s]),
                                   stream="panel" if (multistream and cf[s] == 0) else "update",
                                   waits=[], record=False))
            if multistream and len(esrc):
                gs, gd = gid_of_task[esrc], gid_of_task[edst]
                st_code = np.array([0 if g["stream"] == "panel" else 1 for g in groups], dtype=np.int64)
                sel = st_code[gs] != st_code[gd]
                if sel.any():
                    pairs = np.unique(np.stack([gd[sel], gs[sel]], 1), axis=0)
                    # per destination group, only the latest source group of the other stream matters
                    last = {}
                    for d, s_ in pairs:
                        if s_ > last.get(int(d), -1):
                            last[int(d)] = int(s_)
                    for d, s_ in last.items():
                        groups[d]["waits"].append(s_)
                        groups[s_]["record"] = True
            all_items = items
            nitems_total = len(items)
        dev_items = None
        if device.type == "cuda" and nitems_total:
            host = torch.from_numpy(all_items.view(np.uint8).copy()).pin_memory()
            dev_items = host.to(device, non_blocking=True)
            self._host_items = host
        self.dev_items = dev_items

        # ---------------- dataflow exchanges (parallel.p2p): one per (issue point, phase, dtype),
        # planned identically on every rank; each rank keeps only the peers it has traffic with
        transport = None
        if xrows is not None and len(xrows):
            from ..parallel.p2p import Transport, Xfer, first_after
            transport = Transport(ctx, self.name, lambda: self._bases)
            lk, ll, lw = self._local_access
            wk_me, wl_me = lk[lw], ll[lw]

            def tref(keys, home=False):
                b, o, l = resolve(np.asarray(keys, dtype=np.int64), home)
                out = []
                for i, k in enumerate(keys):
                    M = self.mats[int(k) >> _MID_SHIFT]
                    gm, gn = (int(k) >> _M_SHIFT) & _MASK22, int(k) & _MASK22
                    if M.storage == STORAGE_TILE:
                        # full physical tile: kernels may use storage past a ragged edge
                        # (TSTRF writes one pivot per panel column into an IPIV tile)
                        rows, cols = M.mb, M.nb
                    else:
                        rows, cols = min(M.mb, M.lm - gm * M.mb), min(M.nb, M.ln - gn * M.nb)
                    out.append((int(b[i]), int(o[i]), int(l[i]), rows, cols, M.mb))
                return out

            mid_dt = np.array([dtypes.index(M.dtype) for M in self.mats], dtype=np.int64)
            xdt = mid_dt[xrows[:, 2] >> _MID_SHIFT]
            # global order: issue point, write-backs before fetches, dtype, then peers / key
            gkey = np.stack([xrows[:, 4], 1 - xrows[:, 5], xdt], 1)
            order = np.lexsort((xrows[:, 2], xrows[:, 1], xrows[:, 0], gkey[:, 2], gkey[:, 1], gkey[:, 0]))
            xrows, gkey = xrows[order], gkey[order]
            brk = np.nonzero((gkey[1:] != gkey[:-1]).any(1))[0] + 1
            starts = np.concatenate([[0], brk])
            ends = np.concatenate([brk, [len(xrows)]])
            transport.n_global = len(starts)
            for xid, (a, b_) in enumerate(zip(starts, ends)):
                rows = xrows[a:b_]
                sm = rows[rows[:, 0] == me]
                rm = rows[rows[:, 1] == me]
                if not len(sm) and not len(rm):
                    continue
                dt = dtypes[int(gkey[a, 2])]
                point = int(gkey[a, 0])
                wb = gkey[a, 1] == 0
                sends, recvs = defaultdict(list), defaultdict(list)
                # loopback: a fetch is sent from the home storage, a write-back received into it
                if len(sm):
                    for (dst_r, k), ref in zip(sm[:, [1, 2]].tolist(), tref(sm[:, 2], loop and not wb)):
                        sends[dst_r].append(ref)
                if len(rm):
                    for (src_r, k), ref in zip(rm[:, [0, 2]].tolist(), tref(rm[:, 2], loop and wb)):
                        recvs[src_r].append(ref)
                x = Xfer(xid, dt, nbe_of[dt], sends, recvs, label=f"{'w' if wb else 'f'}@{point}")
                need = None
                if len(rm):
                    if wb:   # write-back into my storage: first later level of mine touching the tile
                        nx = first_after(lk, ll, rm[:, 2], np.full(len(rm), point), nlev)
                        nx = nx[nx >= 0]
                        need = int(nx.min()) if len(nx) else None
                    else:
                        need = int(rm[:, 3].min())
                guard = None
                if len(sm):      # first later level of mine overwriting a tile this exchange packs
                    gx = first_after(wk_me, wl_me, sm[:, 2], np.full(len(sm), point), nlev)
                    gx = gx[gx >= 0]
                    guard = int(gx.min()) if len(gx) else None
                transport.add(x, point, need, guard)
        self.transport = transport
        self._bases = bases
        prog = _DagProgram(self, nlev, groups, transport, dtype, device, multistream)
        tp.task(self.name, "update", prog.run)
        tp.dag = prog
        tp.transport = transport
        return tp.finish_build()


    def _write_dot(self, path, ops, modes, kid, level, max_tasks: int = 20000):
        """Append this DAG (tasks as nodes labelled kind(m,n), RAW/WAR/WAW edges, ranked by
        level) to a DOT file -- the ``--dot`` / ``parsec_dot`` dump of the reference."""
        rt = _lib_rt()
        n = len(kid)
        if rt is None or n > max_tasks:
            with open(path, "a") as f:
                f.write(f"// {self.name}: {n} tasks, not dumped (limit {max_tasks})\n")
            return
        _, _, esrc, edst = rt.dag_schedule(ops, modes)
        ex = np.array([self.kinds[k].exec_role for k in range(len(self.kinds))])[kid]
        key = ops[np.arange(n), ex]
        name = self.name.replace('"', "")
        with open(path, "a") as f:
            f.write(f'digraph "{name}" {{\n  rankdir=TB; node [shape=box, fontsize=9];\n')
            for t in range(n):
                k = int(key[t])
                nm = self.kinds[int(kid[t])].name
                m, c = (k >> _M_SHIFT) & _MASK22, k & _MASK22
                f.write(f'  t{t} [label="{nm}({m},{c})\\nL{int(level[t])}"];\n')
            for a, b in zip(esrc.tolist(), edst.tolist()):
                f.write(f"  t{a} -> t{b};\n")
            f.write("}\n")


class _DagProgram:
    def __init__(self, dag: TileDAG, nlev, groups, transport, dtype, device, multistream):
        self.dag = dag
        self.nlev = nlev
        self.groups = groups
        self.by_level = defaultdict(list)
        for i, g in enumerate(groups):
            self.by_level[g["level"]].append(i)
        self.transport = transport
        self.dtype, self.device = dtype, device
        self.multistream = multistream
        self.nlaunch = len(groups)

    def _launch(self, g, dev_items, stream_ptr, stream_obj=None):
        with trace.span(self.dag.ctx, g["K"].name, "dag", stream_obj,
                        {"level": g["level"], "tasks": g["n"], "dag": self.dag.name}):
            self._launch_now(g, dev_items, stream_ptr, stream_obj)

    def _launch_now(self, g, dev_items, stream_ptr, stream_obj=None):
        K = g["K"]
        if K.body is not None:
            self._run_bodies(g, stream_obj)
            return
        if dev_items is not None:
            K.gpu(dev_items.data_ptr() + g["start"] * DAG_ITEM.itemsize, g["n"], stream_ptr, g["emax"])
        else:
            for refs, e in zip(g["cpu_refs"], g["ext"]):
                K.cpu(refs, (int(e[0]), int(e[1]), int(e[2])))

    def _run_bodies(self, g, stream_obj):
        """DTD task class: one call per task on tile views (tensor views of tile storage)."""
        K = g["K"]
        pyargs = g["pyargs"] or [()] * g["n"]

        def go():
            for refs, shp, pa in zip(g["cpu_refs"], g["shapes"], pyargs):
                views = []
                for (base, off, ld), (r, c) in zip(refs, shp):
                    views.append(None if base is None else torch.as_strided(base, (r, c), (1, ld), off))
                K.body(*views, *pa)
        if stream_obj is not None:
            with torch.cuda.stream(stream_obj):
                go()
        else:
            go()

    def run(self):
        dag = self.dag
        dev_items = dag.dev_items
        if self.multistream and dev_items is not None:
            return self._run_streams(dev_items)
        stream = sobj = None
        if self.device.type == "cuda":
            from ..ops import _lib
            stream = _lib.stream_ptr()
            sobj = torch.cuda.current_stream(self.device)
        tr = self.transport
        if tr is not None:
            tr.start(sobj)
        for L in range(self.nlev):
            if tr is not None:
                tr.before(L, sobj)
            for gi in self.by_level.get(L, ()):
                self._launch(self.groups[gi], dev_items, stream)
            if tr is not None:
                tr.after(L, sobj)
        if tr is not None:
            tr.finish(sobj)

    def _run_streams(self, dev_items):
        """Dataflow over two streams: zero-slack (critical-path) groups on a
        high-priority stream, bulk groups on the other; cross-stream group
        dependencies become event waits."""
        ctx = self.dag.ctx
        cur = torch.cuda.current_stream(ctx.device)
        streams = {"panel": ctx.streams["panel"], "update": ctx.streams["update"]}
        start = torch.cuda.Event()
        start.record(cur)
        for s in streams.values():
            s.wait_event(start)
        events = {}
        for gi, g in enumerate(self.groups):
            s = streams[g["stream"]]
            for w in g["waits"]:
                s.wait_event(events[w])
            self._launch(g, dev_items, s.cuda_stream, s)
            if g["record"]:
                ev = torch.cuda.Event()
                ev.record(s)
                events[gi] = ev
        for s in streams.values():
            ev = torch.cuda.Event()
            ev.record(s)
            cur.wait_event(ev)


from ..parallel.p2p import copy_tiles  # noqa: E402,F401  (re-export)
