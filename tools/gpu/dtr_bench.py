"""DTR Cholesky vs the stream-program engine on one MI355X (same matrix, same check).

  python tools/gpu/dtr_bench.py [N ...] [--engine dtr|stream] [--reps R]
"""
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

import dplasma_amd as dp  # noqa: E402


def run(N, engine, reps=2, check=True):
    os.environ["DPLASMA_POTRF_ENGINE"] = engine
    ctx = dp.init()
    A = dp.block_cyclic(ctx, torch.float64, 512, 512, N, N)
    dp.dplghe(ctx, float(N), dp.dplasmaLower, A, 3872)
    A0 = A.data.clone()
    t0 = time.perf_counter()
    tp = dp.dpotrf_New(ctx, dp.dplasmaLower, A)
    enq = time.perf_counter() - t0
    ts = []
    for _ in range(reps + 1):
        A.data.copy_(A0)
        tp.info.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tp.run(ctx)
        info = tp.complete(ctx)
        ts.append(time.perf_counter() - t0)
    t = min(ts[1:])
    ok, res = None, float("nan")
    if check:
        Ar = A.like()
        Ar.data.copy_(A0)
        ok, res = dp.check_potrf(ctx, dp.dplasmaLower, A, Ar)
        del Ar
    print(f"[****] TIME(s) {t:10.5f} : dpotrf N= {N} NB= 512 engine= {engine:6s}: {tp.flops / t / 1e9:10.1f} gflops "
          f"info={info} check={ok} res={res:.2e} enq={enq:.2f}s", flush=True)
    del A, A0, tp
    torch.cuda.empty_cache()


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("N", type=int, nargs="*")
    ap.add_argument("--engine", default=None, help="dtr | stream (default: both)")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--no-check", action="store_true")
    a = ap.parse_args()
    for N in a.N or [8192, 16384, 32768]:
        for eng in ((a.engine,) if a.engine else ("dtr", "stream")):
            run(N, eng, a.reps, not a.no_check)


if __name__ == "__main__":
    main()
