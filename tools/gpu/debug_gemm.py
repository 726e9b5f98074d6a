import sys, os
sys.path.insert(0, os.getcwd())
import torch
import dplasma_amd as dp
g = dp.init(device="cuda:0"); c = dp.Context(device="cpu")
def run(ta, tb, M, N, K, NB, dt=torch.float64, rep=3):
    am, an = (M, K) if ta == 111 else (K, M)
    bm, bn = (K, N) if tb == 111 else (N, K)
    for r in range(rep):
        res = []
        for ctx in (g, c):
            A = dp.block_cyclic(ctx, dt, NB, NB, am, an); B = dp.block_cyclic(ctx, dt, NB, NB, bm, bn)
            C = dp.block_cyclic(ctx, dt, NB, NB, M, N)
            dp.plrnt(ctx, A, 3872); dp.plrnt(ctx, B, 4674); dp.plrnt(ctx, C, 2873)
            dp.gemm(ctx, ta, tb, 0.51, A, B, -0.42, C)
            res.append(C.to_dense_local())
        d = (res[0] - res[1]).abs()
        bad = (d > 1e-9).nonzero()
        print(ta, tb, M, N, K, NB, "rep", r, "maxerr %.3e" % d.max().item(), "nbad", bad.shape[0],
              "rows", sorted(set(bad[:, 0].tolist()))[:8], "cols", sorted(set(bad[:, 1].tolist()))[:8], flush=True)
run(112, 112, 106, 283, 97, 56)
run(111, 111, 106, 283, 97, 56)
run(112, 111, 106, 283, 97, 56)
run(111, 112, 106, 283, 97, 56)
run(112, 112, 106, 283, 97, 64)
run(112, 112, 128, 256, 128, 64)
