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
  Other tiles it touches are fetched into a per-rank slot arena before the
  level (cached per tile version, so a panel's V/T tiles are fetched once per
  rank, not once per update) and tiles it modifies are written back to their
  home after the level.  Each level's traffic is ONE ``all_to_all_single``
  (RCCL p2p over xGMI), planned identically on every rank from replicated
  metadata; levels without traffic do no collective at all.

Items carry absolute device addresses (``DAG_ITEM``, 96 bytes: six operand
slots, layout of ``QrItem`` in ``csrc/kernels/qr.hip``) so one launch can mix tiles living in
descriptor storage and in the slot arena.  All items are built and uploaded
once at compile time ("ENQ" phase, excluded from timing as in
``tests/common.h:252-277``).
"""
from __future__ import annotations

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

    def add(self, K: Kind, ops, ext, pyargs=None):
        """Append tasks of kind K in program order.

        ops: (n, len(K.roles)) tile keys (-1 for an unused optional role); ext: (n, 3) ints;
        pyargs: optional per-task tuples of Python values passed to a ``body`` kind."""
        ops = np.atleast_2d(np.asarray(ops, dtype=np.int64))
        ext = np.atleast_2d(np.asarray(ext, dtype=np.int32))
        if ops.size == 0:
            return
        if ops.shape[1] != len(K.roles) or ext.shape != (ops.shape[0], 3):
            raise ValueError(f"{K.name}: bad task array shapes {ops.shape} {ext.shape}")
        if pyargs is not None and len(pyargs) != len(ops):
            raise ValueError("one pyargs tuple per task")
        kid = self.kind(K)
        self._chunks.append((kid, ops, ext, list(pyargs) if pyargs is not None else None))
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
    def compile(self) -> Taskpool:
        ctx = self.ctx
        me, world = ctx.rank, ctx.world
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
        p = 0
        for k, o, e, pa in self._chunks:
            n = len(o)
            K = self.kinds[k]
            ops[p:p + n, :o.shape[1]] = o
            for r, (_, md, _) in enumerate(K.roles):
                modes[p:p + n, r] = np.where(o[:, r] >= 0, md, 0)
            kid[p:p + n] = k
            ext[p:p + n] = e
            if pa is not None:
                if pyargs_all is None:
                    pyargs_all = [()] * ntask
                pyargs_all[p:p + n] = pa
            p += n
        self._chunks = []
        names = [K.name for K in self.kinds]
        tp.simulation_date = lambda cost=None: simulation_date(ops, modes, kid, names, cost)
        rt = _lib_rt()
        # single process on a GPU: dataflow over two streams (critical path / bulk)
        multistream = world == 1 and ctx.device.type == "cuda" and rt is not None and MULTISTREAM
        crit = None
        if multistream:
            level, blevel, esrc, edst = rt.dag_schedule(ops, modes)
            depth = level.astype(np.int64) + blevel
            crit = (depth.max() - depth) <= CRIT_SLACK
        else:
            level = rt.dag_levels(ops, modes) if rt is not None else _levels_py(ops, modes)
        nlev = int(level.max()) + 1
        dot = getattr(ctx, "dot_file", None)
        if dot and me == 0:
            self._write_dot(dot, ops, modes, kid, level)
        # executor rank per task
        exec_key = ops[np.arange(ntask), np.array([self.kinds[k].exec_role for k in range(len(self.kinds))])[kid]]
        exe = self._home(exec_key) if world > 1 else np.zeros(ntask, dtype=np.int64)

        # ---------------- remote-tile plan (identical on every rank)
        fetch_at = defaultdict(list)   # level -> rows (src, dst, key)
        wback_at = defaultdict(list)
        slot_of: Dict[int, int] = {}
        if world > 1:
            used = modes > 0
            t_idx, r_idx = np.nonzero(used)
            akeys = ops[t_idx, r_idx]
            home = self._home(akeys)
            aexe = exe[t_idx]
            rem = home != aexe
            if rem.any():
                ver = rt.dag_versions(ops, modes) if rt is not None else _versions_py(ops, modes)
                t_r, r_r = t_idx[rem], r_idx[rem]
                k_r, h_r, e_r = akeys[rem], home[rem], aexe[rem]
                v_r = ver[t_r, r_r].astype(np.int64)
                w_r = (modes[t_r, r_r] & 2) > 0
                l_r = level[t_r].astype(np.int64)
                order = np.lexsort((l_r, k_r, e_r))
                t_r, k_r, h_r, e_r, v_r, w_r, l_r = (x[order] for x in (t_r, k_r, h_r, e_r, v_r, w_r, l_r))
                first = np.ones(len(k_r), dtype=bool)
                first[1:] = (k_r[1:] != k_r[:-1]) | (e_r[1:] != e_r[:-1])
                have = np.empty(len(k_r), dtype=np.int64)
                have[1:] = v_r[:-1] + w_r[:-1]
                need = first | (v_r != np.where(first, -1, have))
                for i in np.nonzero(need)[0]:
                    fetch_at[int(l_r[i])].append((int(h_r[i]), int(e_r[i]), int(k_r[i])))
                for i in np.nonzero(w_r)[0]:
                    wback_at[int(l_r[i])].append((int(e_r[i]), int(h_r[i]), int(k_r[i])))
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

        def resolve(keys):
            """keys (n,) -> (base index, element offset, ld) arrays for this rank."""
            keys = np.asarray(keys, dtype=np.int64)
            mid = (keys >> _MID_SHIFT).astype(np.int64)
            bidx = mid.copy()
            off = np.zeros(len(keys), dtype=np.int64)
            ld = np.zeros(len(keys), dtype=np.int32)
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

        # ---------------- my launches, grouped by (level, critical first, kind prio, kind)
        mine_t = np.nonzero(exe == me)[0] if world > 1 else np.arange(ntask)
        prio = np.array([self.kinds[k].prio for k in range(len(self.kinds))])[kid[mine_t]]
        cflag = (~crit[mine_t]).astype(np.int64) if crit is not None else np.zeros(len(mine_t), dtype=np.int64)
        order = np.lexsort((mine_t, kid[mine_t], prio, cflag, level[mine_t]))
        mine_t = mine_t[order]
        groups = []  # execution order: dict(K, start, n, cpu_refs, ext, emax, level, stream)
        all_items = []
        nitems_total = 0
        if len(mine_t):
            lv, kk = level[mine_t], kid[mine_t]
            cf = cflag[order]
            brk = np.nonzero((lv[1:] != lv[:-1]) | (kk[1:] != kk[:-1]) | (cf[1:] != cf[:-1]))[0] + 1
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

        # ---------------- exchange plans (one all_to_all per level, phase and dtype)
        def xplan(rows, nbe):
            """rows: (src, dst, key) -> my send keys, my receive keys, split sizes (elements)."""
            rows = sorted(rows, key=lambda x: (x[0], x[1], x[2]))
            sends = [r for r in rows if r[0] == me]
            recvs = [r for r in rows if r[1] == me]
            sc = [0] * world
            rc = [0] * world
            for s_, d_, _ in sends:
                sc[d_] += nbe
            for s_, d_, _ in recvs:
                rc[s_] += nbe
            return [k for (_, _, k) in sends], [k for (_, _, k) in recvs], sc, rc

        def copy_plan(keys, nbe):
            """Tile copies between their current place (home storage | arena) and a buffer."""
            from ..ops.batch import TileBatch
            groups = {}
            if not keys:
                return []
            b, o, l = resolve(np.array(keys, dtype=np.int64))
            for i, k in enumerate(keys):
                M = self.mats[k >> _MID_SHIFT]
                gm, gn = (k >> _M_SHIFT) & _MASK22, k & _MASK22
                if M.storage == STORAGE_TILE:
                    # full physical tile: kernels may use storage past a ragged edge
                    # (TSTRF writes one pivot per panel column into an IPIV tile)
                    rows, cols = M.mb, M.nb
                else:
                    rows = min(M.mb, M.lm - gm * M.mb)
                    cols = min(M.nb, M.ln - gn * M.nb)
                g = groups.setdefault((int(b[i]), int(l[i]), M.mb), TileBatch())
                g.add(int(o[i]), rows, cols, b_off=i * nbe)
            return [(bi, ldx, mb, tb.finalize()) for (bi, ldx, mb), tb in groups.items()]

        xch = {}
        for L in range(nlev):
            for phase, rows in (("f", fetch_at.get(L)), ("w", wback_at.get(L))):
                if not rows:
                    continue
                plans = []
                for dt in dtypes:
                    r_dt = [r for r in rows if mat_dt[r[2] >> _MID_SHIFT] == dt]
                    if not r_dt:
                        continue
                    pk, uk, sc, rc = xplan(r_dt, nbe_of[dt])
                    plans.append((dt, copy_plan(pk, nbe_of[dt]), copy_plan(uk, nbe_of[dt]), sc, rc))
                xch[(L, phase)] = plans
        self._bases = bases
        prog = _DagProgram(self, nlev, groups, xch, dtype, device, multistream)
        tp.task(self.name, "update", prog.run)
        tp.dag = prog
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
    def __init__(self, dag: TileDAG, nlev, groups, xch, dtype, device, multistream):
        self.dag = dag
        self.nlev = nlev
        self.groups = groups
        self.by_level = defaultdict(list)
        for i, g in enumerate(groups):
            self.by_level[g["level"]].append(i)
        self.xch = xch
        self.dtype, self.device = dtype, device
        self.multistream = multistream
        self.nlaunch = len(groups)

    def _exchange(self, plans, level=-1):
        with trace.span(self.dag.ctx, f"{self.dag.name}:exchange", "comm", args={"level": level}):
            self._exchange_now(plans)

    def _exchange_now(self, plans):
        bases = self.dag._bases
        for dt, pack, unpack, sc, rc in plans:
            sendbuf = torch.empty(sum(sc), dtype=dt, device=self.device)
            recvbuf = torch.empty(sum(rc), dtype=dt, device=self.device)
            for bi, ld, mb, tb in pack:   # tile (base, off, ld) -> sendbuf[i*nbe] (ld = mb)
                copy_tiles(bases[bi], ld, sendbuf, mb, tb, to_b=True)
            # every rank joins: the plan exists on all ranks whenever the level has this traffic
            dist.all_to_all_single(recvbuf, sendbuf, output_split_sizes=rc, input_split_sizes=sc)
            for bi, ld, mb, tb in unpack:  # recvbuf[i*nbe] -> tile
                copy_tiles(bases[bi], ld, recvbuf, mb, tb, to_b=False)

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
        stream = None
        if self.device.type == "cuda":
            from ..ops import _lib
            stream = _lib.stream_ptr()
        for L in range(self.nlev):
            x = self.xch.get((L, "f"))
            if x is not None:
                self._exchange(x, L)
            for gi in self.by_level.get(L, ()):
                self._launch(self.groups[gi], dev_items, stream)
            x = self.xch.get((L, "w"))
            if x is not None:
                self._exchange(x, L)

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


def copy_tiles(A, lda, B, ldb, tb, to_b: bool):
    """Copy the tiles of a TileBatch (a_off in A, b_off in B) A -> B (to_b) or B -> A.

    Floating-point tiles use the batched copy kernel; integer tiles (pivot
    vectors) are tiny and copied with tensor views."""
    from ..constants import dplasmaNoTrans
    from ..ops import tile_ops as ops
    from ..ops.batch import TileBatch
    tb.finalize()
    if A.dtype.is_floating_point or A.dtype.is_complex:
        if to_b:
            ops.geadd(0, dplasmaNoTrans, 1.0, A, lda, 0.0, B, ldb, tb, copy=True)
            return
        sw = getattr(tb, "_swapped", None)
        if sw is None:
            sw = TileBatch()
            for it in tb.items:
                sw.add(int(it["b_off"]), int(it["m"]), int(it["n"]), b_off=int(it["a_off"]))
            sw.finalize()
            tb._swapped = sw
        ops.geadd(0, dplasmaNoTrans, 1.0, B, ldb, 0.0, A, lda, sw, copy=True)
        return
    for it in tb.items:
        m, n = int(it["m"]), int(it["n"])
        a = torch.as_strided(A, (m, n), (1, lda), int(it["a_off"]))
        b = torch.as_strided(B, (m, n), (1, ldb), int(it["b_off"]))
        (b if to_b else a).copy_(a if to_b else b)
