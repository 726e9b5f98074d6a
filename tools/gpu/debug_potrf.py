import sys, os
sys.path.insert(0, os.getcwd())
import torch
import dplasma_amd as dp
g = dp.init(device="cuda:0"); c = dp.Context(device="cpu")
for (N, NB) in [(1024, 256), (2048, 512), (4096, 512)]:
    outs = []
    for ctx in (g, c):
        A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N); dp.plghe(ctx, float(N), dp.dplasmaLower, A, 3)
        info = dp.potrf(ctx, dp.dplasmaLower, A)
        outs.append(A.to_dense_local().tril())
    d = (outs[0] - outs[1]).abs()
    bad = (d > 1e-9).nonzero()
    print("potrf", N, NB, "info", info, "maxerr", d.max().item(), "first bad", bad[:3].tolist(), "nbad", bad.shape[0], flush=True)
    # tile-level error map
    mt = N // NB
    emap = [[int(d[i*NB:(i+1)*NB, j*NB:(j+1)*NB].max().item() > 1e-9) for j in range(mt)] for i in range(mt)]
    for row in emap: print("".join(map(str, row)))
