"""Tracing / profiling: per-rank timelines of every batched launch and exchange.

Reference: PaRSEC profiling as driven by the tests (``--enable-prof-trace`` ->
``parsec_profiling_start()`` in ``SYNC_TIME_START``, ``tests/common_timing.h:25-44``;
run metadata via ``PROFILING_SAVE_dINFO/iINFO``, ``tests/common.h:198-231``;
``DPLASMA_TRACE_KERNELS`` -> ``printlog`` per kernel call, ``src/dplasmajdf.h:21-31``;
``--dot`` DAG dumps, ``tests/common.c:390-437``).

MI355X design: the unit of work is a *batched launch* (one kernel over all
ready tiles of one kind), so that is what gets traced.  On the GPU a span is a
pair of timing HIP events recorded on the launch's own stream (the panel and
update streams show up as separate tracks, making their overlap visible); on
the CPU it is wall-clock time.  Nothing synchronises while recording; the
events are resolved once in :meth:`Tracer.finalize`.  Output is Chrome trace
JSON (chrome://tracing, Perfetto) with one process per rank, plus a per-name
summary table.  Enable with ``dp.profiling_start(ctx)`` or
``DPLASMA_PROFILE=<file.json>`` in the environment (written at ``dp.fini``).
``DPLASMA_TRACE_KERNELS=1`` prints one line per launch as it is issued.
"""
from __future__ import annotations

import json
import os
import sys
import time
from collections import defaultdict
from contextlib import contextmanager
from typing import Dict, List, Optional

import torch

TRACE_KERNELS = os.environ.get("DPLASMA_TRACE_KERNELS", "0") not in ("", "0")


class Tracer:
    def __init__(self, ctx):
        self.ctx = ctx
        self.rank = ctx.rank
        self.gpu = ctx.is_gpu
        self.meta: Dict[str, object] = {}
        self._open: List[tuple] = []     # (name, cat, track, start, end, args)
        self.events: List[dict] = []
        self._t0 = time.perf_counter()
        self._ev0 = None
        if self.gpu:
            self._ev0 = torch.cuda.Event(enable_timing=True)
            self._ev0.record(torch.cuda.current_stream(ctx.device))

    # ------------------------------------------------------------------ recording
    def _track_of(self, stream) -> str:
        if stream is None:
            return "host"
        for name, s in getattr(self.ctx, "streams", {}).items():
            if s.cuda_stream == stream.cuda_stream:
                return name
        return f"stream{stream.cuda_stream:x}"

    @contextmanager
    def span(self, name: str, cat: str = "task", stream=None, args: Optional[dict] = None, gpu: bool = True):
        if self.gpu and gpu:
            s = stream if stream is not None else torch.cuda.current_stream(self.ctx.device)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(s)
            try:
                yield
            finally:
                e1.record(s)
                self._open.append((name, cat, self._track_of(s), e0, e1, args))
        else:
            t0 = time.perf_counter()
            try:
                yield
            finally:
                self._open.append((name, cat, "host", t0, time.perf_counter(), args))

    def save_info(self, key: str, value):
        """PROFILING_SAVE_dINFO / iINFO analogue: run metadata stored with the trace."""
        self.meta[key] = value

    # ------------------------------------------------------------------ output
    def finalize(self):
        if self.gpu and self._open:
            torch.cuda.synchronize(self.ctx.device)
        for name, cat, track, a, b, args in self._open:
            if isinstance(a, float):
                ts, dur = (a - self._t0) * 1e6, (b - a) * 1e6
            else:
                ts = self._ev0.elapsed_time(a) * 1e3
                dur = a.elapsed_time(b) * 1e3
            ev = {"name": name, "cat": cat, "ph": "X", "pid": self.rank, "tid": track, "ts": ts, "dur": dur}
            if args:
                ev["args"] = args
            self.events.append(ev)
        self._open.clear()
        return self

    def summary(self) -> Dict[str, dict]:
        self.finalize()
        out = defaultdict(lambda: {"count": 0, "total_us": 0.0, "max_us": 0.0})
        for e in self.events:
            r = out[e["name"]]
            r["count"] += 1
            r["total_us"] += e["dur"]
            r["max_us"] = max(r["max_us"], e["dur"])
        return dict(out)

    def print_summary(self, file=sys.stdout, top: int = 30):
        rows = sorted(self.summary().items(), key=lambda kv: -kv[1]["total_us"])[:top]
        print(f"{'name':48s} {'count':>7s} {'total(ms)':>11s} {'max(us)':>10s}", file=file)
        for n, r in rows:
            print(f"{n[:48]:48s} {r['count']:7d} {r['total_us'] / 1e3:11.3f} {r['max_us']:10.1f}", file=file)

    def dump(self, path: str, gather: bool = True):
        """Write a Chrome trace (all ranks' events gathered on rank 0 when distributed)."""
        self.finalize()
        events = list(self.events)
        meta = dict(self.meta)
        if gather and self.ctx.world > 1:
            import torch.distributed as dist
            allev = [None] * self.ctx.world
            dist.all_gather_object(allev, events)
            events = [e for lst in allev for e in lst]
            if self.rank != 0:
                return None
        for r in sorted({e["pid"] for e in events}):
            events.append({"name": "process_name", "ph": "M", "pid": r, "args": {"name": f"rank {r}"}})
        with open(path, "w") as f:
            json.dump({"traceEvents": events, "otherData": meta, "displayTimeUnit": "ms"}, f)
        return path


# ----------------------------------------------------------------------------- helpers used by the runtime
@contextmanager
def _null():
    yield


def span(ctx, name, cat="task", stream=None, args=None, gpu=True):
    """Span on ctx's tracer if profiling is on (cheap no-op otherwise)."""
    tr = getattr(ctx, "profiling", None) if ctx is not None else None
    if TRACE_KERNELS:
        print(f"[dplasma_amd r{getattr(ctx, 'rank', 0)}] {cat}: {name} {args or ''}", file=sys.stderr, flush=True)
    if tr is None:
        return _null()
    return tr.span(name, cat, stream, args, gpu)


def profiling_start(ctx) -> Tracer:
    ctx.profiling = Tracer(ctx)
    return ctx.profiling


def profiling_stop(ctx, path: Optional[str] = None) -> Optional[Tracer]:
    tr = getattr(ctx, "profiling", None)
    ctx.profiling = None
    if tr is not None and path:
        tr.dump(path)
    return tr
