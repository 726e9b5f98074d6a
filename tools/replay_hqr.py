#!/usr/bin/env python3
"""Rank replay of the distributed hierarchical QR (BASELINE config 4: dgeqrf HQR M=N=65536 NB=256 on
a P x Q grid) on ONE GPU -- the HQR counterpart of tools/replay_potrf.py.

Compiles the exact ``geqrf_param_New`` program of rank r (the stacked-domain engine, models/qr_panel.py:
its TS domains, its TT kills with their partners, the V/T row broadcasts, the pairwise partial-W sums)
on a context dressed as that rank and runs it with every exchange replaced by the replay backend's
timing model (``ReplayBackend.sync``: a delay kernel of ``lat + critical-link bytes / bw`` on a
communication stream that the compute stream waits for; the bytes are not moved -- the kernels are
data-independent in run time).  Remote producers are assumed to reach a panel when this rank does
(optimistic-symmetric), so the worst rank's span estimates the job's time.

usage: python tools/replay_hqr.py -N 65536 --nb 256 --grid 2x4 --ranks all [--bw 50 --lat 15]
       [--llvl 1 --hlvl 1 --a 0 --domino -1 --tsrr 0]   (a = 0: one TS domain per process row)
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import dplasma_amd as dp  # noqa: E402
from dplasma_amd.parallel import comm  # noqa: E402
from dplasma_amd.utils.flops import flops  # noqa: E402


def _potrf_tool():
    spec = importlib.util.spec_from_file_location("replay_potrf", os.path.join(ROOT, "tools", "replay_potrf.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def replay_rank(base, P, Q, rank, N, NB, IB, tree_args, steps, fake_rank_context):
    ctx = fake_rank_context(base, P, Q, rank)
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N, name="A")
    dp.plrnt(ctx, A, 3872)
    A0 = A.data.clone()
    TS = dp.block_cyclic(ctx, torch.float64, IB, NB, A.mt * IB, N, name="TS")
    TT = dp.block_cyclic(ctx, torch.float64, IB, NB, A.mt * IB, N, name="TT")
    llvl, hlvl, a, domino, tsrr = tree_args
    tree = dp.hqr_init(dp.dplasmaNoTrans, A, llvl, hlvl, a or -(-A.mt // P), P, domino, tsrr)
    t0 = time.perf_counter()
    tp = dp.geqrf_param_New(ctx, tree, A, TS, TT)
    t_enq = time.perf_counter() - t0
    gpu = ctx.is_gpu
    times = []
    for s in range(steps + 1):
        A.data.copy_(A0)
        if gpu:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        tp.run(ctx)
        if gpu:
            torch.cuda.synchronize()
        if s > 0 or steps == 0:
            times.append(time.perf_counter() - t0)
    del A, A0, TS, TT, tp
    if gpu:
        torch.cuda.empty_cache()
    return min(times), t_enq


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-N", type=int, default=65536)
    ap.add_argument("--nb", type=int, default=256)
    ap.add_argument("--ib", type=int, default=32)
    ap.add_argument("--grid", default="2x4")
    ap.add_argument("--ranks", default="all")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--bw", type=float, default=50.0)
    ap.add_argument("--lat", type=float, default=15.0)
    ap.add_argument("--comm-wg", type=int, default=4)
    ap.add_argument("--llvl", type=int, default=1)
    ap.add_argument("--hlvl", type=int, default=1)
    ap.add_argument("--a", type=int, default=0)
    ap.add_argument("--domino", type=int, default=-1)
    ap.add_argument("--tsrr", type=int, default=0)
    args = ap.parse_args()
    m = _potrf_tool()
    P, Q = map(int, args.grid.lower().split("x"))
    base = dp.init(device="cuda:0" if torch.cuda.is_available() else "cpu")
    be = m.ReplayBackend(base.device, args.bw, args.lat, args.comm_wg)
    comm.set_backend(be)
    ranks = range(P * Q) if args.ranks == "all" else [int(x) for x in args.ranks.split(",")]
    fl = flops("d", "geqrf", args.N, args.N)
    res = {}
    targs = (args.llvl, args.hlvl, args.a, args.domino, args.tsrr)
    for r in ranks:
        t, enq = replay_rank(base, P, Q, r, args.N, args.nb, args.ib, targs, args.steps, m.fake_rank_context)
        res[r] = t
        print(f"rank {r} ({r // Q},{r % Q}): {t * 1e3:9.2f} ms   enq {enq:.2f} s", flush=True)
    worst = max(res.values())
    ideal = fl / (78.6e12 * P * Q)
    out = {"op": "geqrf_param (HQR)", "N": args.N, "NB": args.nb, "IB": args.ib, "grid": f"{P}x{Q}",
           "tree": {"llvl": args.llvl, "hlvl": args.hlvl, "a": args.a, "domino": args.domino, "tsrr": args.tsrr},
           "bw_GBs": args.bw, "lat_us": args.lat, "worst_ms": round(worst * 1e3, 2), "ideal_ms": round(ideal * 1e3, 2),
           "pct_peak": round(100 * ideal / worst, 1), "tflops_job": round(fl / worst / 1e12, 1),
           "per_rank_ms": {str(k): round(v * 1e3, 2) for k, v in res.items()},
           "comm": {k: (round(v, 1) if isinstance(v, float) else v) for k, v in be.stats.items()}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
