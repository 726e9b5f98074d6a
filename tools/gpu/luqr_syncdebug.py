"""Hybrid LU-QR (dgetrf_qrf) with the step loop issued under torch's sync-debug "error" mode: any host
synchronisation inside the factorisation raises.  Prints the time of the factorisation (python
tools/gpu/luqr_syncdebug.py N NB [criteria alpha])."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

import dplasma_amd as dp  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    NB = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    crit = int(sys.argv[3]) if len(sys.argv) > 3 else dp.DEFAULT_CRITERIUM
    alpha = float(sys.argv[4]) if len(sys.argv) > 4 else 1.0
    ctx = dp.init(device="cuda:0")
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    ib = 32
    TS = dp.block_cyclic(ctx, torch.float64, ib, NB, A.mt * ib, N)
    TT = dp.block_cyclic(ctx, torch.float64, ib, NB, A.mt * ib, N)
    IP = dp.qrf_ipiv_descriptor(ctx, A)
    tree = dp.hqr_init(dp.dplasmaNoTrans, A, 1, -1, -1, 1, -1, 0)   # the testing CLI's defaults (p = 1)
    for rep in range(2):
        dp.plrnt(ctx, A, 3872)
        lu_tab = [0] * A.mt
        tp = dp.getrf_qrf_New(ctx, tree, A, IP, TS, TT, crit, alpha, lu_tab)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.cuda.set_sync_debug_mode("error")
        try:
            tp.run(ctx)
        finally:
            torch.cuda.set_sync_debug_mode("default")
        info = tp.complete(ctx)
        t = time.perf_counter() - t0
        fl = 2.0 * N ** 3 / 3.0
        print(f"run {rep}: N={N} NB={NB} crit={crit} alpha={alpha}: {t:.3f} s  {fl / t / 1e12:.2f} TF/s  info={info}  "
              f"LU steps {sum(lu_tab)}/{len(lu_tab)}  (issued under sync-debug 'error')", flush=True)


if __name__ == "__main__":
    main()
