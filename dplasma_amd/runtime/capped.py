"""Memory-capped execution of any tile DAG: host-resident matrices through a bounded device tile arena.

Reference: the PaRSEC device memory manager every DPLASMA task class runs on -- a fixed pool of
device blocks (``--mca device_cuda_memory_number_of_blocks``, the ``1gpu_lowmem`` tests of
``tests/Testings.cmake:147``), tiles staged in on demand, written back and evicted LRU when the pool
is full, for POTRF, GEQRF, GETRF_INCPIV ... alike.

Design (one process; matrices whose storage is on the host while the context drives a GPU, or any
DAG when ``DPLASMA:GPU:number_of_blocks`` caps the arena):

* the tasks run in dependency-level order (program order inside a level);
* consecutive tasks of one kind and level form a *batch* as long as the distinct tiles they touch fit
  in the arena -- each batch is still ONE batched launch of the kind's kernel, its items pointing
  into the arena;
* the arena is an LRU cache simulated at compile time: every batch pins its tiles, missing tiles
  are loaded (dirty victims written back first), written tiles become dirty, and everything dirty
  goes home at the end.  The resulting op list (write-back / load / launch) is replayed on the
  compute stream at run time, so a run is deterministic and needs no host bookkeeping.

``CappedStats`` (loads, write-backs, launches, peak slots) is attached to the taskpool.
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass

import numpy as np
import torch

from ..constants import STORAGE_TILE


@dataclass
class CappedStats:
    nslots: int = 0
    loads: int = 0
    writebacks: int = 0
    launches: int = 0
    tasks: int = 0


def arena_slots(ctx, mats) -> int:
    """Arena size in tiles: DPLASMA:GPU:number_of_blocks, else 80 % of the free device memory."""
    n = ctx.info.get_int("DPLASMA:GPU:number_of_blocks", 0)
    if n > 0:
        return n
    nbe = max(M.mb * M.nb * M.data.element_size() for M in mats)
    free = torch.cuda.mem_get_info(ctx.device)[0] if ctx.is_gpu else 1 << 34
    total = sum(M.mt * M.nt for M in mats)
    return max(8, min(total, int(0.8 * free) // nbe))


def wanted(ctx, mats) -> bool:
    """Capped mode: one process, and a host-resident matrix on a GPU context or an explicit cap."""
    if ctx.world != 1:
        return False
    if ctx.info.get_int("DPLASMA:GPU:number_of_blocks", 0) > 0:
        return True
    return ctx.is_gpu and any(M.data.device.type == "cpu" for M in mats)


def compile_capped(dag, tp, ops, modes, kid, ext, pyargs_all, level, item_dtype, sub_all=None):
    """Fill ``tp`` with one task replaying the capped schedule of the DAG (see module docstring)."""
    from .dag import _MASK22, _M_SHIFT, _MID_SHIFT, _DagProgram
    ctx = dag.ctx
    device = ctx.device
    mats = dag.mats
    nslots = arena_slots(ctx, mats)
    ntask = len(kid)
    order = np.lexsort((np.arange(ntask), level))
    dtypes = sorted({M.dtype for M in mats}, key=str)
    nbe_of = {dt: max(M.mb * M.nb for M in mats if M.dtype == dt) for dt in dtypes}
    arenas = {dt: torch.zeros(nslots * nbe_of[dt], dtype=dt, device=device) for dt in dtypes}

    def host_view(key):
        M = mats[key >> _MID_SHIFT]
        gm, gn = (key >> _M_SHIFT) & _MASK22, key & _MASK22
        off = int(dag._local_offsets(np.array([key], dtype=np.int64))[0])
        if M.storage == STORAGE_TILE:
            rows, cols = M.mb, M.nb      # the full physical tile (kernels may use it past a ragged edge)
        else:
            rows, cols = min(M.mb, M.lm - gm * M.mb), min(M.nb, M.ln - gn * M.nb)
        return torch.as_strided(M.data, (rows, cols), (1, M.ld), off), M.mb

    def dev_view(key, slot):
        M = mats[key >> _MID_SHIFT]
        hv, ld = host_view(key)
        return torch.as_strided(arenas[M.dtype], tuple(hv.shape), (1, ld), slot * nbe_of[M.dtype])

    # ---- batches: same kind and level, distinct tiles <= nslots (per dtype)
    batches = []
    cur, cur_tiles, cur_k, cur_l = [], set(), None, None
    for t in order.tolist():
        keys = [int(x) for x in ops[t] if x >= 0]
        k, lv = int(kid[t]), int(level[t])
        if len(set(keys)) > nslots:
            raise RuntimeError(f"{dag.name}: a task touches {len(set(keys))} tiles, the arena holds {nslots}")
        new = cur_tiles | set(keys)
        if cur and (k != cur_k or lv != cur_l or len(new) > nslots or dag.kinds[k].body is not None):
            batches.append(cur)
            cur, new = [], set(keys)
        cur.append(t)
        cur_tiles, cur_k, cur_l = new, k, lv
    if cur:
        batches.append(cur)

    # ---- LRU simulation -> op list
    slot = OrderedDict()          # key -> slot, least recently used first (per dtype pools)
    free = {dt: list(range(nslots - 1, -1, -1)) for dt in dtypes}
    dirty = set()
    plan = []                     # ("wb", key, slot) / ("ld", key, slot) / ("go", group index)
    groups, items_all = [], []
    stats = CappedStats(nslots=nslots)
    esz = {dt: torch.empty(0, dtype=dt).element_size() for dt in dtypes}
    for b in batches:
        need = OrderedDict()
        for t in b:
            for x in ops[t]:
                if x >= 0:
                    need[int(x)] = True
        for key in need:
            if key in slot:
                slot.move_to_end(key)
                continue
            dt = mats[key >> _MID_SHIFT].dtype
            if not free[dt]:
                victim = next((v for v in slot if v not in need and mats[v >> _MID_SHIFT].dtype == dt), None)
                if victim is None:
                    raise RuntimeError(f"{dag.name}: tile arena of {nslots} slots exhausted by one batch")
                vs = slot.pop(victim)
                if victim in dirty:
                    plan.append(("wb", victim, vs))
                    dirty.discard(victim)
                    stats.writebacks += 1
                free[dt].append(vs)
            s = free[dt].pop()
            slot[key] = s
            plan.append(("ld", key, s))
            stats.loads += 1
        for t in b:
            for r in range(ops.shape[1]):
                if ops[t, r] >= 0 and modes[t, r] & 2:
                    dirty.add(int(ops[t, r]))
        # the batch's items (arena addresses) / CPU refs
        K = dag.kinds[int(kid[b[0]])]
        seg = np.zeros(len(b), dtype=item_dtype)
        cpu_refs = []
        for i, t in enumerate(b):
            refs = []
            for r, (_, _, sl) in enumerate(K.roles):
                key = int(ops[t, r])
                if key < 0:
                    refs.append((None, 0, 0))
                    continue
                M = mats[key >> _MID_SHIFT]
                ar = arenas[M.dtype]
                off = slot[key] * nbe_of[M.dtype]
                if sub_all is not None:
                    off += int(sub_all[t, r, 0]) + int(sub_all[t, r, 1]) * M.mb
                seg[f"p{sl}"][i] = ar.data_ptr() + off * esz[M.dtype]
                seg[f"ld{sl}"][i] = M.mb
                refs.append((ar, off, M.mb))
            cpu_refs.append(refs)
        ex = ext[np.array(b)]
        seg["m"], seg["n"], seg["k"] = ex[:, 0], ex[:, 1], ex[:, 2]
        start = sum(len(x) for x in items_all)
        items_all.append(seg)
        shapes = [[dag._tile_shape(int(ops[t, r])) for r in range(len(K.roles))] for t in b] if K.body else None
        groups.append(dict(K=K, start=start, n=len(b), cpu_refs=cpu_refs, ext=ex,
                           pyargs=[pyargs_all[t] for t in b] if pyargs_all is not None else None, shapes=shapes,
                           emax=tuple(int(x) for x in ex.max(0)), level=int(level[b[0]]), stream="update",
                           waits=[], record=False))
        plan.append(("go", len(groups) - 1))
        stats.launches += 1
        stats.tasks += len(b)
    for key in list(slot):
        if key in dirty:
            plan.append(("wb", key, slot[key]))
            stats.writebacks += 1
    items = np.concatenate(items_all) if items_all else np.zeros(0, dtype=item_dtype)
    dev_items = None
    if device.type == "cuda" and len(items):
        dev_items = torch.from_numpy(items.view(np.uint8).copy()).to(device)
    prog = _DagProgram(dag, 1, groups, None, mats[0].dtype, device, False)

    def run():
        stream = None
        if device.type == "cuda":
            from ..ops import _lib
            stream = _lib.stream_ptr()
        for op in plan:
            if op[0] == "go":
                prog._launch(groups[op[1]], dev_items, stream)
            elif op[0] == "ld":
                dev_view(op[1], op[2]).copy_(host_view(op[1])[0])
            else:
                host_view(op[1])[0].copy_(dev_view(op[1], op[2]))

    tp.task(dag.name + "[capped]", "update", run)
    tp.capped = stats
    tp.dag = prog
    tp._arenas = arenas
    tp._dev_items = dev_items
    return tp.finish_build()
