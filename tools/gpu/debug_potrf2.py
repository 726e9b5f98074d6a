import sys, os
sys.path.insert(0, os.getcwd())
import torch
import dplasma_amd as dp
from dplasma_amd.models import check as chk, aux
g = dp.init(device="cuda:0"); c = dp.Context(device="cpu")
for uplo in (122, 121):
  for (N, NB) in [(378, 93), (186, 93), (93, 93), (99, 93)]:
    outs = {}
    for name, ctx in (("g", g), ("c", c)):
        A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N); dp.plghe(ctx, float(N), uplo, A, 3872)
        A0 = A.like(); dp.lacpy(ctx, dp.dplasmaUpperLower, A, A0)
        info = dp.potrf(ctx, uplo, A)
        F = A.to_dense_local()
        R = A0.like(); aux.lacpy(ctx, uplo, A0, R); chk._herm_fill(ctx, uplo, R)
        H = R.to_dense_local()
        ok, res = dp.check_potrf(ctx, uplo, A, A0)
        outs[name] = (F, H, res, info)
    tri = (lambda x: x.tril()) if uplo == 122 else (lambda x: x.triu())
    dF = (tri(outs["g"][0]) - tri(outs["c"][0])).abs()
    dH = (outs["g"][1] - outs["c"][1]).abs()
    bad = (dF > 1e-9).nonzero()
    print(uplo, N, NB, "info", outs["g"][3], outs["c"][3], "factor err %.2e" % dF.max().item(), "bad", bad[:3].tolist(),
          "herm err %.2e" % dH.max().item(), "res g/c", outs["g"][2], outs["c"][2], flush=True)
