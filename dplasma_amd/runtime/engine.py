"""Bridge to the native C++ task engine (``lib/_dplasma_rt*.so``).

``run_gpu(tp, ctx)`` hands a taskpool's task list to the engine, which owns
the HIP events / stream waits for cross-stream edges and the optional
per-task timestamps; task bodies stay Python callables that enqueue kernels.
"""
from __future__ import annotations

_RT = None
_TRIED = False


def module():
    global _RT, _TRIED
    if not _TRIED:
        _TRIED = True
        try:
            from ..lib import _dplasma_rt as rt  # type: ignore
            _RT = rt
        except Exception:
            _RT = None
    return _RT


def available() -> bool:
    return module() is not None and hasattr(module(), "run_stream_program")


def run_gpu(tp, ctx):
    rt = module()
    streams = {name: s.cuda_stream for name, s in ctx.streams.items()}
    import torch
    cur = torch.cuda.current_stream(ctx.device).cuda_stream
    rt.run_stream_program([(t.stream, t.fn, t.deps, t.needs_event) for t in tp.tasks], streams, cur,
                          tp.trace is not None)
