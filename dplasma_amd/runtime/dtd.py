"""Dynamic task discovery (DTD) front end: ``insert_task`` on tiles.

Reference surface (SURVEY.md §2.2 "DTD"): ``parsec_dtd_taskpool_new``,
``parsec_dtd_create_task_class`` + ``parsec_dtd_task_class_add_chore``,
``parsec_dtd_insert_task(_with_task_class)``, ``PARSEC_DTD_TILE_OF``,
``PARSEC_INPUT/INOUT/OUTPUT/AFFINITY/VALUE/SCRATCH``,
``parsec_dtd_data_flush(_all)`` -- used by ``src/dtd_wrappers/zpotrf.c:151-171``
and ``tests/testing_zpotrf_dtd.c:74-311``.

Design: inserted tasks go, in program order, into a *window*; their tile
arguments become DAG roles (access mode from the flags) and every other
argument is passed through by value.  When the window holds ``window`` tasks
(``parsec_dtd_window_size``; ``DPLASMA_DTD_WINDOW``, default 4096) it is
compiled into a :class:`TileDAG` and launched at once -- on the GPU the
launches are asynchronous, so insertion of the next window overlaps the
execution of the previous one, as PaRSEC's DTD engine runs tasks while the
application is still inserting.  Consecutive windows are ordered by the
stream (and, distributed, by each window's write-backs), so program-order
semantics hold across window boundaries.  Each task body is called with tensor
views of its tiles on the tile's device -- a body that calls dplasma_amd tile
kernels (or any torch op) runs on the GPU stream the runtime chose.  Tasks
execute on the rank owning the AFFINITY tile (default: the first written
tile), exactly the DTD placement rule.

``data_flush(tile | M)`` launches the pending window: every tile it wrote is
back at its home, and the remote copies of windows older than the last two are
released (``parsec_dtd_data_flush``: the bound on memory).  Bodies may insert
further tasks into the taskpool they run in ("untied" tasks,
``tests/testing_zpotrf_dtd_untied.c``): those land after everything inserted
so far and run in a later window.  A task WITHOUT tile arguments has no data to
follow, so -- as in PaRSEC -- it runs on every rank where it is inserted, at once
(``insert_task`` calls its body); its insertions are therefore identical on every
rank and untied insertion works on any number of processes.  A body that returns
:data:`AGAIN` (``PARSEC_HOOK_RETURN_AGAIN``) is called again after the tasks it
inserted so far have been launched -- the reference inserter's way of bounding the
window.  Tile-carrying bodies that insert tasks run only on their executing rank,
so they are limited to one process.

A task class may instead provide a batched ``Kind`` (``task_class(kind=...)``):
then all ready tasks of that class in a level become one kernel launch.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional

import numpy as np

from .dag import Kind, R, RW, TileDAG, W

INPUT, OUTPUT, INOUT = R, W, RW
AFFINITY = 8       # flag OR-ed into a tile argument: run the task where this tile lives
VALUE = 16         # scalar passed by value (wrapper marker; plain Python values are values too)
SCRATCH = 32       # temporary passed by value (the body allocates it)
PUSHOUT = 64       # accepted for API parity: tiles are always written back to their home
AGAIN = "PARSEC_HOOK_RETURN_AGAIN"   # body return value: call me again once my insertions are launched


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
    """``parsec_dtd_taskpool_new`` analogue: insert tasks, then :meth:`wait` (or :meth:`execute`)."""

    KEEP = 2   # windows whose remote copies stay alive (older ones are released on flush)

    def __init__(self, ctx, name: str = "dtd", window: Optional[int] = None):
        import os
        self.ctx = ctx
        self.name = name
        # window = 0: deferred -- nothing runs until compile() / wait() (the _New taskpools)
        w = int(os.environ.get("DPLASMA_DTD_WINDOW", 4096)) if window is None else int(window)
        self.window = w if w > 0 else float("inf")
        self._new_dag()
        self._kinds: Dict[tuple, Kind] = {}
        self.ntasks = 0
        self.flops = 0.0
        self.pending = 0
        self.windows_run = 0          # windows launched so far (insertion continues meanwhile)
        self._live: List[tuple] = []  # (compiled taskpool, completion event) of recent windows
        self._running = False
        self._on_complete: List[Callable] = []

    def _new_dag(self):
        self.dag = TileDAG(self.ctx, f"{self.name}[{getattr(self, 'windows_run', 0)}]")
        self.dag.no_dtd = True

    def task_class(self, name: str, body: Optional[Callable] = None, kind: Optional[Kind] = None) -> TaskClass:
        """A task class with a Python ``body`` (called per task with its tile views and values) or a
        batched tile ``kind``: its tasks then pass exactly the kind's roles as tile arguments (same
        access modes) and their (m, n, k) extents as the only value."""
        return TaskClass(name, body, kind)

    def _kind_for(self, tc: TaskClass, modes: tuple, affinity: int) -> Kind:
        key = (id(tc), modes, affinity)
        K = self._kinds.get(key)
        if K is None:
            roles = tuple((f"t{i}", md, min(i, 5)) for i, md in enumerate(modes))
            K = Kind(f"dtd:{tc.name}:{len(self._kinds)}", roles, affinity, None, None, body=tc.body)
            self._kinds[key] = K
        return K

    def _batched_kind(self, tc: TaskClass, modes: tuple, affinity: int) -> Kind:
        K = tc.kind
        if len(modes) != len(K.roles) or any(md != r[1] for md, r in zip(modes, K.roles)):
            raise ValueError(f"DTD task class {tc.name}: tile access modes {modes} do not match kind {K.name}")
        if affinity == K.exec_role:
            return K
        key = (id(tc), "exec", affinity)
        Ka = self._kinds.get(key)
        if Ka is None:
            Ka = self._kinds[key] = dataclasses.replace(K, name=f"{K.name}@{affinity}", exec_role=affinity)
        return Ka

    def insert_task(self, fn, *args, name: Optional[str] = None, flops: float = 0.0, priority: int = 0):
        """Insert one task.  ``args`` mixes tile arguments ``(tile_of(A, m, n), INPUT|INOUT|OUTPUT[|AFFINITY])``
        (or a bare TileRef, read-only) and plain values; the body is called as
        ``fn(*tile_views, *values)`` with tiles first, in argument order.  ``priority`` (the
        reference's per-insert priority, tests/testing_zpotrf_dtd.c): among the tasks of a window that
        are ready together (one DAG level), higher priorities issue first (the stream -- critical path
        or bulk -- still follows the task's slack in the DAG)."""
        if self._running and self.ctx.world > 1:
            raise RuntimeError("DTD: a task with tile arguments inserts only on its executing rank; insert from "
                               "a task without tiles (it runs on every rank) on more than one process")
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
            if tc.kind is not None or tc.body is None:
                raise ValueError("a DTD task without tile arguments needs a Python body")
            self._run_local(tc, values)
            return
        if affinity is None:
            written = [i for i, md in enumerate(modes) if md & 2]
            affinity = written[0] if written else 0
        keys = [int(self.dag.keys(t.M, t.m, t.n)) for t in tiles]
        if tc.kind is not None:
            # batched tile kind: the values are the task's (m, n, k) extents; every ready task of the
            # class in a level becomes one launch
            K = self._batched_kind(tc, tuple(modes), affinity)
            ext = [int(x) for x in (values[0] if values else (0, 0, 0))]
            self.dag.add(K, [keys], [ext], prio=[int(priority)])
        else:
            K = self._kind_for(tc, tuple(modes), affinity)
            self.dag.add(K, [keys], [[0, 0, 0]], pyargs=[tuple(values)], prio=[int(priority)])
        self.ntasks += 1
        self.pending += 1
        self.flops += flops
        if self.pending >= self.window and not self._running:
            self._launch()

    def _run_local(self, tc: TaskClass, values):
        """A task without data: run its body here, on every rank (AGAIN: launch what it inserted, then
        call it again)."""
        self.ntasks += 1
        while tc.body(*values) == AGAIN:
            if self.window == float("inf"):
                continue      # deferred taskpool: nothing runs before compile(); keep inserting
            self._launch()

    # ------------------------------------------------------------------ execution
    def _launch(self):
        """Compile the pending window and start it (asynchronous on the GPU)."""
        while self.pending:
            dag, self.pending = self.dag, 0
            self.windows_run += 1
            self._new_dag()
            tp = dag.compile()
            self._running = True
            try:
                tp.run(self.ctx)
            finally:
                self._running = False
            ev = None
            if self.ctx.is_gpu:
                import torch
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(self.ctx.device))
            self._live.append((tp, ev))
            if self.pending < self.window:   # tasks inserted by bodies wait for the next trigger
                break

    def _release(self, keep: int):
        while len(self._live) > keep:
            tp, ev = self._live.pop(0)
            if ev is not None:
                ev.synchronize()
            tp.destruct()

    def data_flush(self, tile=None):
        """parsec_dtd_data_flush(_all): launch what is pending (the data goes home) and release the
        remote copies of older windows.  Deferred taskpools (window 0) flush at the end of their run."""
        if self.window == float("inf"):
            return 0
        self._launch()
        self._release(self.KEEP)
        return 0

    data_flush_all = data_flush

    def on_complete(self, fn: Callable):
        self._on_complete.append(fn)

    def wait(self):
        """parsec_dtd_taskpool_wait: run everything inserted (including tasks inserted by bodies)."""
        while self.pending:
            self._launch()
        if self.ctx.is_gpu:
            import torch
            torch.cuda.current_stream(self.ctx.device).synchronize()
        self._release(0)
        res = None
        for fn in self._on_complete:
            r = fn()
            if r is not None:
                res = r
        return res

    def compile(self):
        """The pending tasks as one compiled (re-runnable) taskpool: the _New form of a DTD algorithm."""
        dag, self.pending = self.dag, 0
        self._new_dag()
        dag.flops = self.flops
        tp = dag.compile()
        tp.ntasks = self.ntasks
        return tp

    def execute(self):
        return self.wait()


def taskpool_new(ctx, name: str = "dtd", window: Optional[int] = None) -> DTDTaskpool:
    return DTDTaskpool(ctx, name, window)
