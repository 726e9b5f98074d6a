"""Rate of the four transpose variants of the batched MFMA GEMM engine (k_gemm_full) on trailing-update
shapes: 32 x 32 output tiles of 512, k = 512 (LU / QR panel width) and k = 2048 (POTRF deferred block).
Lower POTRF runs NT, upper POTRF TN, LU NN, the QR apply TN + NN."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import dplasma_amd as dp  # noqa: E402
from dplasma_amd.ops import tile_ops as ops  # noqa: E402
from dplasma_amd.ops.batch import GemmBatch  # noqa: E402

N_, T_ = dp.dplasmaNoTrans, dp.dplasmaTrans


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


def main():
    ctx = dp.init(device="cuda:0")
    nb, g = 512, 32
    n = nb * g
    for kd in (1, 4):
        K = nb * kd
        # A holds op(A) tiles m x K (N) or K x m (T); B holds K x n (N) or n x K (T): one n x K panel each
        A = dp.block_cyclic(ctx, torch.float64, nb, nb, n, K)
        At = dp.block_cyclic(ctx, torch.float64, nb, nb, K, n)
        C = dp.block_cyclic(ctx, torch.float64, nb, nb, n, n)
        dp.plrnt(ctx, A, 1)
        dp.plrnt(ctx, At, 2)
        for ta in (N_, T_):
            for tb in (N_, T_):
                gb = GemmBatch()
                for nn in range(g):
                    for mm in range(g):
                        kp = []
                        for q in range(kd):
                            ao = A.offset(mm, q) if ta == N_ else At.offset(q, mm)
                            bo = At.offset(q, nn) if tb == N_ else A.offset(nn, q)
                            kp.append((ao, bo, nb))
                        gb.add(C.offset(mm, nn), nb, nb, kp)
                srcA = A if ta == N_ else At
                srcB = At if tb == N_ else A
                t = timeit(lambda: ops.gemm(ta, tb, -1.0, srcA.data, srcA.ld, srcB.data, srcB.ld, 1.0, C.data, C.ld,
                                            gb))
                fl = 2.0 * n * n * K
                name = ("N" if ta == N_ else "T") + ("N" if tb == N_ else "T")
                print(f"gemm {name} tiles={g}x{g} k={K}: {t * 1e3:8.2f} ms  {fl / t / 1e12:6.2f} TF/s", flush=True)


if __name__ == "__main__":
    main()
