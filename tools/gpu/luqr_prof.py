"""Host profile of the hybrid LU-QR (getrf_qrf) on one GPU: cProfile of one factorisation, top functions by
cumulative and by own time (python tools/gpu/luqr_prof.py N NB)."""
import cProfile
import pstats
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

import dplasma_amd as dp  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    NB = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    ctx = dp.init(device="cuda:0")
    for rep in range(2):
        A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
        dp.plrnt(ctx, A, 3872)
        ib = 32
        TS = dp.block_cyclic(ctx, torch.float64, ib, NB, A.mt * ib, N)
        TT = dp.block_cyclic(ctx, torch.float64, ib, NB, A.mt * ib, N)
        IP = dp.qrf_ipiv_descriptor(ctx, A)
        tree = dp.hqr_init(dp.dplasmaNoTrans, A, 1, -1, -1, 1, -1, 0)   # the testing CLI's defaults
        lu_tab = [0] * A.mt
        tp = dp.getrf_qrf_New(ctx, tree, A, IP, TS, TT, 0, 1.0, lu_tab)
        torch.cuda.synchronize()
        pr = cProfile.Profile()
        pr.enable()
        t0 = time.perf_counter()
        tp.execute(ctx)
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        pr.disable()
        print(f"run {rep}: {t:.3f} s  lu_tab={lu_tab}", flush=True)
    st = pstats.Stats(pr)
    st.sort_stats("cumulative").print_stats(30)
    st.sort_stats("tottime").print_stats(20)


if __name__ == "__main__":
    main()
