#!/usr/bin/env python3
"""Per-kernel micro-benchmarks (device time via HIP events), for tuning.

python tools/kbench.py [potrf|trsm|gemm|all]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import dplasma_amd as dp
from dplasma_amd.ops import tile_ops as ops
from dplasma_amd.ops.batch import GemmBatch, TileBatch


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


def bench_potrf(ctx, nbs=(128, 256, 512)):
    for nb in nbs:
        A = dp.block_cyclic(ctx, torch.float64, nb, nb, nb, nb)
        dp.plghe(ctx, float(nb), dp.dplasmaLower, A, 1)
        A0 = A.data.clone()
        info = torch.zeros(1, dtype=torch.int32, device=ctx.device)

        def f():
            A.data.copy_(A0)
            ops.potrf_tile(dp.dplasmaLower, A.data, 0, nb, A.ld, info, 0)
        t = timeit(f)
        tc = timeit(lambda: A.data.copy_(A0))
        fl = nb ** 3 / 3
        print(f"potrf_tile nb={nb}: {t - tc:9.1f} us  ({fl / (t - tc) / 1e3:7.1f} GF/s)", flush=True)


def bench_trsm(ctx, nb=512, ntiles=(1, 8, 64)):
    for nt in ntiles:
        T = dp.block_cyclic(ctx, torch.float64, nb, nb, nb, nb)
        dp.plghe(ctx, float(nb), dp.dplasmaLower, T, 1)
        info = torch.zeros(1, dtype=torch.int32, device=ctx.device)
        ops.potrf_tile(dp.dplasmaLower, T.data, 0, nb, T.ld, info, 0)
        B = dp.block_cyclic(ctx, torch.float64, nb, nb, nb * nt, nb)
        dp.plrnt(ctx, B, 2)
        tb = TileBatch()
        for m in range(nt):
            tb.add(0, nb, nb, b_off=B.offset(m, 0))
        t = timeit(lambda: ops.trsm(dp.dplasmaRight, dp.dplasmaLower, dp.dplasmaConjTrans, dp.dplasmaNonUnit, 1.0,
                                    T.data, T.ld, B.data, B.ld, tb))
        fl = nt * nb ** 3
        print(f"trsm RLCN nb={nb} tiles={nt}: {t:9.1f} us ({fl / t / 1e3:7.1f} GF/s)", flush=True)


def bench_gemm(ctx, nb=512, grid=(1, 4, 16, 64)):
    for g in grid:
        n = nb * g
        A = dp.block_cyclic(ctx, torch.float64, nb, nb, n, nb)
        C = dp.block_cyclic(ctx, torch.float64, nb, nb, n, n)
        dp.plrnt(ctx, A, 1)
        gb = GemmBatch()
        for nn in range(g):
            for mm in range(g):
                gb.add(C.offset(mm, nn), nb, nb, [(A.offset(mm, 0), A.offset(nn, 0), nb)])
        t = timeit(lambda: ops.gemm(dp.dplasmaNoTrans, dp.dplasmaConjTrans, -1.0, A.data, A.ld, A.data, A.ld, 1.0,
                                    C.data, C.ld, gb))
        fl = 2.0 * n * n * nb
        print(f"gemm NT tiles={g}x{g} k={nb}: {t:9.1f} us ({fl / t / 1e3:8.1f} GF/s)", flush=True)
    # trailing-update shapes with k aggregated over several panels (deferred updates)
    for kd in (2, 4):
        g = 32
        n = nb * g
        A = dp.block_cyclic(ctx, torch.float64, nb, nb, n, nb * kd)
        C = dp.block_cyclic(ctx, torch.float64, nb, nb, n, n)
        dp.plrnt(ctx, A, 1)
        gb = GemmBatch()
        for nn in range(g):
            for mm in range(g):
                gb.add(C.offset(mm, nn), nb, nb, [(A.offset(mm, q), A.offset(nn, q), nb) for q in range(kd)])
        t = timeit(lambda: ops.gemm(dp.dplasmaNoTrans, dp.dplasmaConjTrans, -1.0, A.data, A.ld, A.data, A.ld, 1.0,
                                    C.data, C.ld, gb))
        fl = 2.0 * n * n * nb * kd
        print(f"gemm NT tiles={g}x{g} k={nb * kd}: {t:9.1f} us ({fl / t / 1e3:8.1f} GF/s)", flush=True)
    # one big multi-k GEMM (SUMMA single rank)
    for n in [int(x) for x in os.environ.get("KBENCH_GEMM_N", "8192,16384").split(",")]:
        A = dp.block_cyclic(ctx, torch.float64, nb, nb, n, n)
        B = dp.block_cyclic(ctx, torch.float64, nb, nb, n, n)
        C = dp.block_cyclic(ctx, torch.float64, nb, nb, n, n)
        dp.plrnt(ctx, A, 1)
        dp.plrnt(ctx, B, 2)
        tp = dp.gemm_New(ctx, dp.dplasmaNoTrans, dp.dplasmaNoTrans, 1.0, A, B, 0.0, C)
        t = timeit(lambda: tp.run(ctx), reps=3)
        print(f"gemm NN {n}^3 nb={nb}: {t:9.1f} us ({2.0 * n ** 3 / t / 1e3:8.1f} GF/s)", flush=True)


if __name__ == "__main__":
    ctx = dp.init(device="cuda:0")
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what in ("potrf", "all"):
        bench_potrf(ctx)
    if what in ("trsm", "all"):
        bench_trsm(ctx)
    if what in ("gemm", "all"):
        bench_gemm(ctx)


def potrf_phases(ctx):
    import ctypes
    from dplasma_amd.ops import _lib
    lib = _lib.load()
    lib.dpl_debug_set_phase_mask.argtypes = [ctypes.c_int]
    for mask, name in [(0xff, "all"), (0, "none"), (1, "stageY"), (2, "a"), (4, "b-chol"), (8, "c-mfma"), (16, "d-write"),
                       (0xff & ~4, "all-but-b"), (0xff & ~2, "all-but-a")]:
        lib.dpl_debug_set_phase_mask(mask)
        for nb in (128, 512):
            A = dp.block_cyclic(ctx, torch.float64, nb, nb, nb, nb)
            dp.plghe(ctx, float(nb), dp.dplasmaLower, A, 1)
            info = torch.zeros(1, dtype=torch.int32, device=ctx.device)
            t = timeit(lambda: ops.potrf_tile(dp.dplasmaLower, A.data, 0, nb, A.ld, info, 0))
            print(f"phases {name:10s} nb={nb}: {t:8.1f} us", flush=True)
    lib.dpl_debug_set_phase_mask(0xff)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "phases":
    potrf_phases(dp.init(device="cuda:0"))
