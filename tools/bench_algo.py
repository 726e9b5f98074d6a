#!/usr/bin/env python3
"""Quick single-GPU timing of one algorithm (factorizations beyond the headline bench).

python tools/bench_algo.py geqrf -N 8192 --nb 256 --ib 32 [--tree hqr] [--runs 2]
Prints the reference-style line ``[****] TIME(s) ... : X gflops``.
"""
import argparse
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch

import dplasma_amd as dp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("op")
    ap.add_argument("-N", type=int, default=8192)
    ap.add_argument("-M", type=int, default=0)
    ap.add_argument("--nb", type=int, default=256)
    ap.add_argument("--ib", type=int, default=32)
    ap.add_argument("--runs", type=int, default=2)
    ap.add_argument("--prec", default="d")
    ap.add_argument("--tree", default="flat")
    ap.add_argument("--qr-a", type=int, default=0, help="HQR TS domain size in tiles (0: one domain per process row)")
    ap.add_argument("--qr-llvl", type=int, default=1, help="HQR low-level tree (0 flat, 1 greedy, 2 fibonacci, 3 binary)")
    ap.add_argument("--qr-hlvl", type=int, default=1, help="HQR high-level tree")
    ap.add_argument("--qr-domino", type=int, default=-1, help="HQR domino (-1: reference auto)")
    ap.add_argument("--qr-tsrr", type=int, default=0, help="HQR round-robin TS killers")
    ap.add_argument("--engine", default="panel", help="QR engine: panel (stacked domains) or tile")
    a = ap.parse_args()
    ctx = dp.init(device="cuda:0")
    from dplasma_amd.models import qr_panel
    qr_panel._ENGINE[0] = a.engine
    dt = {"s": torch.float32, "d": torch.float64, "c": torch.complex64, "z": torch.complex128}[a.prec]
    M = a.M or a.N
    N = a.N
    for r in range(a.runs):
        A = dp.block_cyclic(ctx, dt, a.nb, a.nb, M, N)
        dp.plrnt(ctx, A, 3872)
        if a.op in ("geqrf", "gelqf"):
            TS = dp.block_cyclic(ctx, dt, a.ib, a.nb, A.mt * a.ib, A.nt * a.nb)
            TT = dp.block_cyclic(ctx, dt, a.ib, a.nb, A.mt * a.ib, A.nt * a.nb)
            t0 = time.perf_counter()
            if a.tree == "flat":
                tp = (dp.geqrf_New if a.op == "geqrf" else dp.gelqf_New)(ctx, A, TS)
            else:
                tr_ = dp.dplasmaNoTrans if a.op == "geqrf" else dp.dplasmaConjTrans
                rows = A.mt if a.op == "geqrf" else A.nt
                P_ = ctx.P if a.op == "geqrf" else ctx.Q
                tree = dp.hqr_init(tr_, A, a.qr_llvl, a.qr_hlvl, a.qr_a or -(-rows // P_), P_,
                                   a.qr_domino, a.qr_tsrr)
                tp = (dp.geqrf_param_New if a.op == "geqrf" else dp.gelqf_param_New)(ctx, tree, A, TS, TT)
        elif a.op == "getrf_nopiv":
            dp.plghe(ctx, float(N), dp.dplasmaUpperLower, A, 3872)
            t0 = time.perf_counter()
            tp = dp.getrf_nopiv_New(ctx, A)
        elif a.op == "getrf_ptgpanel":
            IPIV = dp.ptgpanel_ipiv_descriptor(ctx, A)
            t0 = time.perf_counter()
            tp = dp.getrf_ptgpanel_New(ctx, A, IPIV)
        elif a.op == "getrf_incpiv":
            L = dp.incpiv_L_descriptor(ctx, A, a.ib)
            IPIV = dp.incpiv_ipiv_descriptor(ctx, A)
            t0 = time.perf_counter()
            tp = dp.getrf_incpiv_New(ctx, A, L, IPIV)
        elif a.op == "gemm":
            B = dp.block_cyclic(ctx, dt, a.nb, a.nb, N, N)
            C = dp.block_cyclic(ctx, dt, a.nb, a.nb, M, N)
            dp.plrnt(ctx, B, 4674)
            dp.plrnt(ctx, C, 2873)
            t0 = time.perf_counter()
            tp = dp.gemm_New(ctx, dp.dplasmaNoTrans, dp.dplasmaNoTrans, 0.51, A, B, -0.42, C)
        elif a.op == "getrf_1d":
            IPIV = dp.ipiv_descriptor(ctx, A)
            t0 = time.perf_counter()
            tp = dp.getrf_1d_New(ctx, A, IPIV)
        elif a.op in ("herbt", "heev"):
            dp.plghe(ctx, 0.0, dp.dplasmaLower, A, 3872)
            t0 = time.perf_counter()
            if a.op == "herbt":
                tp = dp.herbt_New(ctx, dp.dplasmaLower, a.ib, A, dp.eigen_T(A, a.ib))
            else:
                W = torch.zeros(N, dtype=torch.float64)
                tp = dp.heev_New(ctx, dp.dplasmaNoVec, dp.dplasmaLower, A, W, ib=a.ib)
        elif a.op == "gebrd_ge2gb":
            t0 = time.perf_counter()
            tp = dp.gebrd_ge2gb_New(ctx, a.ib, A)
        else:
            raise SystemExit(f"unknown op {a.op}")
        torch.cuda.synchronize()
        t_enq = time.perf_counter() - t0
        t1 = time.perf_counter()
        tp.run(ctx)
        torch.cuda.synchronize()
        tp.complete(ctx)
        t = time.perf_counter() - t1
        nl = getattr(getattr(tp, "dag", None), "nlaunch", None)
        print(f"[****] TIME(s) {t:12.5f} : {a.op}\tPxQxg= 1 1 1 NB= {a.nb} N= {N} M= {M} : "
              f"{tp.flops / t / 1e9:14.3f} gflops - ENQ {t_enq:.3f}s launches {nl}", flush=True)


if __name__ == "__main__":
    main()
