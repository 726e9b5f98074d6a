#!/usr/bin/env python3
"""One SUMMA-style single-rank DGEMM (N^3, NB=512) run a few times -- PMC/trace target."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

import dplasma_amd as dp

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
ctx = dp.init(device="cuda:0")
nb = 512
A = dp.block_cyclic(ctx, torch.float64, nb, nb, n, n)
B = dp.block_cyclic(ctx, torch.float64, nb, nb, n, n)
C = dp.block_cyclic(ctx, torch.float64, nb, nb, n, n)
dp.plrnt(ctx, A, 1)
dp.plrnt(ctx, B, 2)
tp = dp.gemm_New(ctx, dp.dplasmaNoTrans, dp.dplasmaNoTrans, 1.0, A, B, 0.0, C)
for _ in range(reps):
    tp.run(ctx)
torch.cuda.synchronize()
print("done", flush=True)
if os.environ.get("VENDOR"):
    # calibration only: the vendor library on the same random shape (never used by the framework)
    a = torch.randn(n, n, dtype=torch.float64, device="cuda")
    b = torch.randn(n, n, dtype=torch.float64, device="cuda")
    for _ in range(reps):
        c = a @ b
    torch.cuda.synchronize()
    print("vendor done", flush=True)
