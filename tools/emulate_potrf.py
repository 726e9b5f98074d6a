#!/usr/bin/env python3
"""Model a P x Q grid's distributed DTR Cholesky on ONE MI355X (models/potrf_dtr_dist.py Emulation).

Each XCD runs one rank's share (8 ranks: one XCD each, i.e. 1/8 of a GPU per rank), the ranks' tiles,
receive buffers, W and counters are separate, and the kernel dilates time by P Q: a task's completion
becomes visible (P Q - 1) x its duration after it ends, a strip sent over a rank pair's link (FIFO)
arrives P Q x (lat + bytes / bw) after the link frees.  span / (P Q) is the modelled time of the grid on
P Q GPUs (compute, HBM share, critical-path latency and link time all dilated by the same factor; the
infinity cache is shared by the emulated ranks, which makes the model slightly pessimistic).

  python tools/emulate_potrf.py -N 65536 --grid 2x4 [--bw 50] [--lat 10] [--reps 2] [--check]
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import dplasma_amd as dp  # noqa: E402
from dplasma_amd.models import potrf_dtr_dist as DD  # noqa: E402
from dplasma_amd.utils.flops import flops  # noqa: E402

PEAK = 78.6e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-N", type=int, default=32768)
    ap.add_argument("--grid", default="2x4")
    ap.add_argument("--bw", type=float, default=50.0, help="GB/s per link and direction")
    ap.add_argument("--lat", type=float, default=10.0, help="us per message")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--trace", default=None, help="write the per-task trace (npz)")
    ap.add_argument("--order", default="step", choices=["deadline", "column", "panel", "rowpipe", "step"])
    ap.add_argument("--defer", type=int, default=None)
    a = ap.parse_args()
    P, Q = (int(x) for x in a.grid.lower().split("x"))
    ctx = dp.init()
    em = DD.Emulation(ctx, a.N, P, Q, bw_gbs=a.bw, lat_us=a.lat, trace=a.trace is not None, order=a.order,
                      Dd=a.defer)
    nr = P * Q
    f = flops("d", "potrf", a.N)
    pl = em.plan
    print(f"[emul] N={a.N} grid={P}x{Q} tasks={len(pl.tasks)} sends={pl.nsend} W-sends={pl.nsendw} "
          f"recv tiles/rank={[len(t) for t in pl.recv_tiles]}", flush=True)
    spans = []
    for rep in range(a.reps + 1):
        em.reset()
        s = em.run()
        spans.append(s)
        t = s / nr
        print(f"[emul] rep {rep}: span {s:.4f} s -> {P}x{Q} modelled {t * 1e3:.1f} ms = {f / t / 1e12:.1f} TF/s "
              f"= {100 * f / t / (nr * PEAK):.1f} % of {nr} x 78.6 TF/s (bw {a.bw} GB/s, lat {a.lat} us)", flush=True)
    best = min(spans[1:] if len(spans) > 1 else spans) / nr
    print(f"[****] EMUL {P}x{Q} N={a.N} NB=512 order={a.order} D={em.plan.base.D}: {best * 1e3:.1f} ms {f / best / 1e9:.1f} gflops "
          f"{100 * f / best / (nr * PEAK):.1f} % of peak", flush=True)
    if a.trace:
        import numpy as np
        np.savez(a.trace, trace=em.trace[:4 * len(pl.tasks)].view(-1, 4).cpu().numpy(), owner=pl.owner, type=pl.tasks["type"],
                 k0=pl.tasks["k0"], i=pl.tasks["i"], j=pl.tasks["j"], nk=pl.tasks["nk"], inc=pl.tasks["inc"],
                 req_beg=pl.tasks["req_beg"], nreq=pl.tasks["nreq"], reqs=pl.reqs, nranks=nr)
    if a.check:
        L, A0 = em.assemble()
        del em                      # the per-rank storage, receive buffers and W: the 64k check needs the room
        import gc
        gc.collect()
        torch.cuda.empty_cache()
        ok, res = dp.check_potrf(ctx, dp.dplasmaLower, L, A0)
        print(f"[emul] residual {res:.3e} check={ok}", flush=True)
        if not ok:
            sys.exit(1)


if __name__ == "__main__":
    main()
