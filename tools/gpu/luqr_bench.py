"""Hybrid LU-QR (getrf_qrf) timing on one MI355X for data-dependent criteria (device-decided steps, p = domain period)
against the DEFAULT criterion:

  python tools/gpu/luqr_bench.py [N] [NB] [p]

Prints seconds, GFLOP/s (LU flop count, as the reference tester) and the LU / QR step split per criterion."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

import dplasma_amd as dp  # noqa: E402
from dplasma_amd.models import lu_qr, qrtree  # noqa: E402
from dplasma_amd.utils.flops import flops  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    NB = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    p = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    ib = 32
    ctx = dp.init(device="cuda:0")
    for crit, alpha, name in ((dp.DEFAULT_CRITERIUM, 1.0, "DEFAULT"), (dp.HIGHAM_SUM_CRITERIUM, 1.0, "HIGHAM_SUM"),
                              (dp.HIGHAM_CRITERIUM, 0.02, "HIGHAM"), (dp.MUMPS_CRITERIUM, 1.0, "MUMPS")):
        best = None
        for rep in range(2):
            A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
            dp.plrnt(ctx, A, 3872)
            TS = dp.block_cyclic(ctx, torch.float64, ib, NB, A.mt * ib, N)
            TT = dp.block_cyclic(ctx, torch.float64, ib, NB, A.mt * ib, N)
            IP = dp.qrf_ipiv_descriptor(ctx, A)
            tree = qrtree.hqr_init(dp.dplasmaNoTrans, A, qrtree.GREEDY_TREE, qrtree.FLAT_TREE, p, p)
            tp = lu_qr.getrf_qrf_New(ctx, tree, A, IP, TS, TT, crit, alpha, p=p)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tp.run(ctx)
            tp.complete(ctx)
            torch.cuda.synchronize()
            t = time.perf_counter() - t0
            best = t if best is None else min(best, t)
            tab = list(tp.lu_tab)
            dev = getattr(tp, "devcrit", False)
            del A, TS, TT, IP, tp
            torch.cuda.empty_cache()
        gf = flops("d", "getrf", N, N) / best / 1e9
        print(f"[****] getrf_qrf N={N} NB={NB} p={p} {name:10s}: {best:8.3f} s {gf:10.1f} gflops  LU steps "
              f"{sum(tab)} / {len(tab)}  device-decided={dev}", flush=True)


if __name__ == "__main__":
    main()
