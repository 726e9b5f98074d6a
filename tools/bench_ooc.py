#!/usr/bin/env python3
"""Time the memory-bounded GEMM (host operands) against the device-resident GEMM at one size."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import dplasma_amd as dp  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
NB = 512
g = dp.init(device="cuda:0")
cpu = dp.init(device="cpu")
mats = []
for s in range(3):
    X = dp.TiledMatrix(torch.float64, NB, NB, N, N, device="cpu")
    X.data = X.data.pin_memory()
    dp.plrnt(cpu, X, s + 1)
    mats.append(X)
A, B, C = mats
fl = 2.0 * N ** 3
for r in range(2):
    t = time.perf_counter()
    dp.gemm_gpu(g, dp.dplasmaNoTrans, dp.dplasmaNoTrans, 1.0, A, B, 0.0, C)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(f"[****] TIME(s) {dt:12.5f} : dgemm_gpu (host operands) N= {N} NB= {NB} : {fl / dt / 1e9:14.3f} gflops",
          flush=True)
dA, dB, dC = (dp.block_cyclic(g, torch.float64, NB, NB, N, N) for _ in range(3))
for X, s in zip((dA, dB), (1, 2)):
    dp.plrnt(g, X, s)
for r in range(2):
    torch.cuda.synchronize()
    t = time.perf_counter()
    dp.gemm(g, dp.dplasmaNoTrans, dp.dplasmaNoTrans, 1.0, dA, dB, 0.0, dC)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(f"[****] TIME(s) {dt:12.5f} : dgemm (resident) N= {N} NB= {NB} : {fl / dt / 1e9:14.3f} gflops", flush=True)
