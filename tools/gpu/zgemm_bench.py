"""Complex GEMM engine rate (zgemm.hip) and complex Cholesky (zpotrf) on one MI355X.

  python tools/gpu/zgemm_bench.py [N_gemm] [N_potrf ...]
"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

import dplasma_amd as dp  # noqa: E402
from dplasma_amd.constants import dplasmaNoTrans  # noqa: E402
from dplasma_amd.ops import tile_ops as ops  # noqa: E402
from dplasma_amd.ops.batch import GemmBatch  # noqa: E402


def gemm_rate(N, dt, generic=False, nb=512):
    A = torch.randn(3 * N * N, dtype=dt, device="cuda")
    gb = GemmBatch()
    for i in range(0, N, nb):
        for j in range(0, N, nb):
            gb.add(2 * N * N + i + j * N, nb, nb, [(i, N * N + j * N, N)], 0)
    gb.finalize()
    ops.FORCE_GENERIC_GEMM = generic
    try:
        f = lambda: ops.gemm(dplasmaNoTrans, dplasmaNoTrans, 1.0, A, N, A, N, 0.0, A, N, gb)  # noqa: E731
        f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            f()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 3 / 1e3
    finally:
        ops.FORCE_GENERIC_GEMM = False
    return 8.0 * N ** 3 / t / 1e12, t


def main():
    ng = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    for dt in (torch.complex128, torch.complex64):
        tf, t = gemm_rate(ng, dt)
        tg, _ = gemm_rate(ng, dt, generic=True) if ng <= 8192 else (float("nan"), 0)
        print(f"{dt} gemm {ng}^3: MFMA {tf:7.2f} TF/s ({t * 1e3:.1f} ms)   generic FMA {tg:7.2f} TF/s", flush=True)
    ctx = dp.init()
    for N in [int(a) for a in sys.argv[2:]] or [16384]:
        A = dp.block_cyclic(ctx, torch.complex128, 512, 512, N, N)
        dp.zplghe(ctx, float(N), dp.dplasmaLower, A, 3872)
        A0 = A.data.clone()
        tp = dp.zpotrf_New(ctx, dp.dplasmaLower, A)
        tp.execute(ctx)
        A.data.copy_(A0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        info = tp.execute(ctx)
        t = time.perf_counter() - t0
        fl = tp.flops
        Ar = A.like()
        Ar.data.copy_(A0)
        ok, res = dp.check_potrf(ctx, dp.dplasmaLower, A, Ar)
        print(f"[****] TIME(s) {t:10.5f} : zpotrf N= {N} NB= 512 : {fl / t / 1e9:12.1f} gflops info={info} "
              f"check={ok} res={res:.2e}", flush=True)


if __name__ == "__main__":
    main()
