"""Dynamic task discovery (DTD) front end: ``insert_task`` on tiles.

Reference surface (SURVEY.md §2.2 "DTD"): ``parsec_dtd_taskpool_new``,
``parsec_dtd_create_task_class`` + ``parsec_dtd_task_class_add_chore``,
``parsec_dtd_insert_task(_with_task_class)``, ``PARSEC_DTD_TILE_OF``,
``PARSEC_INPUT/INOUT/OUTPUT/AFFINITY/VALUE/SCRATCH``,
``parsec_dtd_data_flush(_all)`` -- used by ``src/dtd_wrappers/zpotrf.c:151-171``
and ``tests/testing_zpotrf_dtd.c:74-311``.

Design: inserted tasks go, in program order, into a :class:`TileDAG`; their
tile arguments become the DAG roles (access mode from the flags) and every
other argument is passed through by value.  Executing the taskpool runs the
DAG with the dataflow executor (levels, critical-path stream, distributed
fetch/write-back), and each task body is called with tensor views of its
tiles on the tile's device -- so a body that calls dplasma_amd tile kernels
(or any torch op) runs on the GPU stream the runtime chose.  Tasks execute on
the rank owning the AFFINITY tile (default: the first written tile), exactly
the DTD placement rule.

A task class may instead provide a batched ``Kind`` (``task_class(kind=...)``):
then all ready tasks of that class in a level become one kernel launch.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Dict, List, Optional

import numpy as np

from .dag import Kind, R, RW, TileDAG, W

INPUT, OUTPUT, INOUT = R, W, RW
AFFINITY = 8       # flag OR-ed into a tile argument: run the task where this tile lives
VALUE = 16         # scalar passed by value (wrapper marker; plain Python values are values too)
SCRATCH = 32       # temporary passed by value (the body allocates it)
PUSHOUT = 64       # accepted for API parity: tiles are always written back to their home


@dataclass(frozen=True)
class TileRef:
    """PARSEC_DTD_TILE_OF(M, m, n)."""
    M: object
    m: int
    n: int


def tile_of(M, m: int, n: int) -> TileRef:
    return TileRef(M, int(m), int(n))


class TaskClass:
    """A DTD task class: a Python body (and optionally a batched GPU kind)."""

    def __init__(self, name: str, body: Callable, kind: Optional[Kind] = None):
        self.name, self.body, self.kind = name, body, kind


class DTDTaskpool:
    """``parsec_dtd_taskpool_new`` analogue; compile with :meth:`compile` or run with :meth:`execute`."""

    def __init__(self, ctx, name: str = "dtd"):
        self.ctx = ctx
        self.name = name
        self.dag = TileDAG(ctx, name)
        self._kinds: Dict[tuple, Kind] = {}
        self.ntasks = 0
        self.flops = 0.0

    def task_class(self, name: str, body: Callable, kind: Optional[Kind] = None) -> TaskClass:
        return TaskClass(name, body, kind)

    def _kind_for(self, tc: TaskClass, modes: tuple, affinity: int) -> Kind:
        key = (id(tc), modes, affinity)
        K = self._kinds.get(key)
        if K is None:
            roles = tuple((f"t{i}", md, min(i, 5)) for i, md in enumerate(modes))
            K = Kind(f"dtd:{tc.name}:{len(self._kinds)}", roles, affinity, None, None, body=tc.body)
            self._kinds[key] = K
        return K

    def insert_task(self, fn, *args, name: Optional[str] = None, flops: float = 0.0):
        """Insert one task.  ``args`` mixes tile arguments ``(tile_of(A, m, n), INPUT|INOUT|OUTPUT[|AFFINITY])``
        (or a bare TileRef, read-only) and plain values; the body is called as
        ``fn(*tile_views, *values)`` with tiles first, in argument order."""
        tc = fn if isinstance(fn, TaskClass) else TaskClass(name or getattr(fn, "__name__", "task"), fn)
        tiles, modes, values = [], [], []
        affinity = None
        for a in args:
            if isinstance(a, TileRef):
                a = (a, INPUT)
            if isinstance(a, tuple) and len(a) == 2 and isinstance(a[0], TileRef):
                ref, flag = a
                md = flag & 3
                if md == 0:
                    raise ValueError("tile argument needs INPUT, OUTPUT or INOUT")
                if flag & AFFINITY:
                    affinity = len(tiles)
                tiles.append(ref)
                modes.append(md)
            elif isinstance(a, tuple) and len(a) == 2 and a[1] in (VALUE, SCRATCH):
                values.append(a[0])
            else:
                values.append(a)
        if not tiles:
            raise ValueError("a DTD task needs at least one tile argument")
        if affinity is None:
            written = [i for i, md in enumerate(modes) if md & 2]
            affinity = written[0] if written else 0
        K = self._kind_for(tc, tuple(modes), affinity)
        keys = [int(self.dag.keys(t.M, t.m, t.n)) for t in tiles]
        self.dag.add(K, [keys], [[0, 0, 0]], pyargs=[tuple(values)])
        self.ntasks += 1
        self.flops += flops

    def data_flush(self, M=None):
        """parsec_dtd_data_flush(_all): data is always written back to its home
        tile by the end of a run, so this only documents the intent."""
        return 0

    data_flush_all = data_flush

    def compile(self):
        self.dag.flops = self.flops
        tp = self.dag.compile()
        tp.ntasks = self.ntasks
        return tp

    def execute(self):
        return self.compile().execute(self.ctx)


def taskpool_new(ctx, name: str = "dtd") -> DTDTaskpool:
    return DTDTaskpool(ctx, name)
