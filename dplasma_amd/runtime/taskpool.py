"""Taskpools: the executable form of an algorithm (``X_New`` result).

An algorithm is compiled at ``_New`` time into a list of *tasks*; each task
is a coarse unit (one batched kernel launch, one panel kernel, one
collective) bound to a stream class (``panel``/``update``/``aux``) with
explicit dependencies on earlier tasks.  Execution enqueues every task in
program order on its stream, inserting HIP event waits only for
cross-stream edges, so the whole factorisation is queued asynchronously and
the GPU runs ahead of the host (the HIP-native replacement for PaRSEC's
ready-queue dispatch).  The dependency bookkeeping and event
management are done by the loop in ``_run_gpu_py`` (task bodies are Python
callables that enqueue native kernels through ctypes); on CPU tasks simply
run in order.

Issue order: program order by default; a context scheduler policy
(``ctx.scheduler``: the reference's ``-o`` choice -- lfq, ltq, ap, lhq, spq, pbq
(priority first), ip (inverse priority), gd (FIFO), ll (LIFO), rnd) makes the
native ready-queue list scheduler (``csrc/runtime/dag_core.h`` ``list_schedule``)
pick the order in which ready tasks are enqueued, by their ``prio``.  Every
order it produces is a topological order, so stream order plus the cross-stream
events keep the dataflow intact.  Multi-process taskpools always issue in
program order: their communication tasks must reach every rank in the same
order.

Timing protocol (reference ``tests/common.h:252-277``): building the
taskpool is ENQ, ``run`` + ``complete`` is PROG, ``destruct`` is DEST.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence

import numpy as np
import torch

# scheduler names (PaRSEC's -o) -> list_schedule policy codes
SCHED_POLICY = {"": 0, "po": 0, "program": 0, "lfq": 1, "ltq": 1, "ap": 1, "lhq": 1, "spq": 1, "pbq": 1,
                "ip": 2, "gd": 3, "ll": 4, "rnd": 5}


def policy_code(name) -> int:
    key = (name or "").strip().lower()
    if key not in SCHED_POLICY:
        raise ValueError(f"unknown scheduler {name!r} (known: {', '.join(sorted(k for k in SCHED_POLICY if k))})")
    return SCHED_POLICY[key]


@dataclass
class Task:
    tid: int
    name: str
    stream: str
    fn: Callable[[], None]
    deps: List[int] = field(default_factory=list)
    prio: int = 0
    needs_event: bool = False
    comm: Optional[bool] = None       # issues communication (None: unknown -- treated as True)


class Taskpool:
    def __init__(self, name: str, ctx=None):
        self.name = name
        self.ctx = ctx
        self.tasks: List[Task] = []
        self.flops = 0.0
        self._on_complete: List[Callable] = []
        self._on_destruct: List[Callable] = []
        self._result = None
        self.t_enq = time.perf_counter()
        self.t_prog = None
        self.trace = None

    # ------------------------------------------------------------------ build
    def task(self, name: str, stream: str, fn: Callable[[], None], deps: Sequence[Optional[int]] = (),
             prio: int = 0, comm: Optional[bool] = None) -> int:
        """Append a task.  ``comm=False`` declares a compute-only task (it may wait for exchanges that
        its dependencies started, but starts none): on more than one rank only such tasks are
        reordered by a scheduler policy; every other task keeps its program order."""
        tid = len(self.tasks)
        dd = [d for d in deps if d is not None]
        for d in dd:
            if d >= tid:
                raise ValueError("dependencies must point to earlier tasks")
            if self.tasks[d].stream != stream:
                self.tasks[d].needs_event = True
        self.tasks.append(Task(tid, name, stream, fn, dd, prio, comm=comm))
        return tid

    def on_complete(self, fn: Callable):
        self._on_complete.append(fn)

    def on_destruct(self, fn: Callable):
        """Release hook of resources shared with other ranks (called by every rank from destruct)."""
        self._on_destruct.append(fn)

    def finish_build(self):
        self.t_enq = time.perf_counter() - self.t_enq
        return self

    # ------------------------------------------------------------------ execute
    def run(self, ctx=None):
        from ..utils import trace
        ctx = ctx or self.ctx
        with trace.span(ctx, self.name, "taskpool", args={"tasks": len(self.tasks), "gflop": self.flops / 1e9}):
            self._run(ctx)

    def _run(self, ctx):
        t0 = time.perf_counter()
        if ctx is not None and ctx.is_gpu:
            self._run_gpu_py(ctx)
        else:
            from ..utils import trace
            from ..parallel import comm
            for ti in self.issue_order(ctx):
                t = self.tasks[ti]
                comm.LABEL = t.name
                with trace.span(ctx, t.name, "task", gpu=False):
                    t.fn()
        self._t_run = t0

    def issue_order(self, ctx=None) -> List[int]:
        """Task issue order under the context's scheduler policy (see module docstring)."""
        ctx = ctx or self.ctx
        n = len(self.tasks)
        pol = policy_code(getattr(ctx, "scheduler", None)) if ctx is not None else 0
        if pol == 0 or n < 2:
            return list(range(n))
        cache = self.__dict__.setdefault("_orders", {})
        if pol in cache:
            return cache[pol]
        from .dag import _lib_rt
        rt = _lib_rt()
        if rt is None:
            return list(range(n))
        multi = ctx is not None and ctx.world > 1
        deps = [list(t.deps) for t in self.tasks]
        if multi:
            # every rank must issue its communication in the same (program) order: chain the tasks
            # that may communicate; compute-only tasks (comm=False) are free to move by priority
            prev = None
            for t in self.tasks:
                if t.comm is not False:
                    if prev is not None and prev not in deps[t.tid]:
                        deps[t.tid].append(prev)
                    prev = t.tid
        ptr = np.zeros(n + 1, dtype=np.int64)
        for t in self.tasks:
            ptr[t.tid + 1] = len(deps[t.tid])
        ptr = np.cumsum(ptr)
        idx = np.array([d for dl in deps for d in dl], dtype=np.int64)
        prio = np.array([t.prio for t in self.tasks], dtype=np.int32)
        order = [int(x) for x in rt.dag_list_schedule(ptr, idx, prio, pol, int(getattr(ctx, "sched_seed", 0)))]
        cache[pol] = order
        return order

    def _run_gpu_py(self, ctx):
        from ..parallel import comm
        from ..utils import trace
        cur = torch.cuda.current_stream(ctx.device)
        start = torch.cuda.Event()
        start.record(cur)
        used = {t.stream for t in self.tasks}
        for s in used:
            ctx.streams[s].wait_event(start)
        events = {}
        for ti in self.issue_order(ctx):
            t = self.tasks[ti]
            s = ctx.streams[t.stream]
            for d in t.deps:
                if self.tasks[d].stream != t.stream:
                    s.wait_event(events[d])
            comm.LABEL = t.name
            with torch.cuda.stream(s), trace.span(ctx, t.name, "task", s):
                t.fn()
            if t.needs_event:
                ev = torch.cuda.Event()
                ev.record(s)
                events[t.tid] = ev
        for s in used:
            ev = torch.cuda.Event()
            ev.record(ctx.streams[s])
            cur.wait_event(ev)

    def complete(self, ctx=None):
        ctx = ctx or self.ctx
        if ctx is not None and ctx.is_gpu:
            torch.cuda.current_stream(ctx.device).synchronize()
        res = None
        for fn in self._on_complete:
            r = fn()
            if r is not None:
                res = r
        self._result = res
        self.t_prog = time.perf_counter() - getattr(self, "_t_run", time.perf_counter())
        return res

    def execute(self, ctx=None):
        """Blocking run (add + start + wait)."""
        self.run(ctx)
        return self.complete(ctx)

    @property
    def result(self):
        return self._result

    def destruct(self):
        for fn in self.__dict__.get("_on_destruct", []):
            fn()
        self._on_destruct = []
        self.tasks = []
        self._on_complete = []
