import sys, os
sys.path.insert(0, os.getcwd())
import torch
import dplasma_amd as dp
from dplasma_amd.ops import tile_ops as ops
from dplasma_amd.ops.batch import TileBatch
g = dp.init(device="cuda:0"); c = dp.Context(device="cpu")
def run(prec, side, uplo, trans, diag, m, n):
    dt = {"s": torch.float32, "d": torch.float64, "z": torch.complex128}[prec]
    k = m if side == dp.dplasmaLeft else n
    outs = []
    for ctx in (g, c):
        T = dp.block_cyclic(ctx, dt, k, k, k, k); dp.plghe(ctx, float(k), dp.dplasmaUpperLower, T, 11)
        B = dp.block_cyclic(ctx, dt, m, n, m, n); dp.plrnt(ctx, B, 12)
        ops.trsm(side, uplo, trans, diag, 0.7, T.data, T.ld, B.data, B.ld, TileBatch().add(0, m, n, b_off=0))
        outs.append(B.to_dense_local())
    d = (outs[0] - outs[1]).abs()
    bad = (d > 1e-6 * outs[1].abs().max()).nonzero()
    print(prec, side, uplo, trans, diag, m, n, "maxerr", d.max().item(), "nbad", bad.shape[0], "first", bad[:4].tolist())
for prec in "sd":
    for side in (141, 142):
        for uplo in (122, 121):
            for trans in (111, 112):
                run(prec, side, uplo, trans, 131, 150, 93)
run("d", 142, 122, 113, 131, 512, 512)
run("d", 141, 122, 111, 131, 16, 16)
run("d", 141, 122, 111, 131, 32, 4)
run("d", 141, 122, 111, 131, 17, 3)
# potrf tile alone
for N in (16, 32, 100, 512):
    outs = []
    for ctx in (g, c):
        A = dp.block_cyclic(ctx, torch.float64, N, N, N, N); dp.plghe(ctx, float(N), dp.dplasmaLower, A, 3)
        info = torch.zeros(1, dtype=torch.int32, device=A.device)
        ops.potrf_tile(dp.dplasmaLower, A.data, 0, N, A.ld, info, 0)
        outs.append(A.to_dense_local().tril())
    d = (outs[0] - outs[1]).abs()
    print("potrf", N, d.max().item(), (d > 1e-10).nonzero()[:4].tolist())
