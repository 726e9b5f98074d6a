#!/usr/bin/env python3
"""Calibration only: vendor DGEMM (torch.matmul -> rocBLAS/hipBLASLt) TF/s on this MI355X.

Not used by the framework (no vendor BLAS in the compute path); it tells us what fp64
MFMA throughput the card sustains under load (clock/power), i.e. the practical ceiling
our hand-written GEMM engine is measured against.
"""
import torch

torch.manual_seed(0)
for n in (4096, 8192, 16384):
    a = torch.randn(n, n, dtype=torch.float64, device="cuda")
    b = torch.randn(n, n, dtype=torch.float64, device="cuda")
    c = a @ b
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5 if n < 16384 else 3
    s.record()
    for _ in range(reps):
        c = a @ b
    e.record()
    torch.cuda.synchronize()
    t = s.elapsed_time(e) / reps / 1e3
    print(f"vendor dgemm {n}^3: {t*1e3:9.2f} ms  {2*n**3/t/1e12:6.2f} TF/s", flush=True)
# K=512 trailing-update shape: C(16384x16384) -= A(16384x512) B^T
n, k = 16384, 512
a = torch.randn(n, k, dtype=torch.float64, device="cuda")
c = torch.randn(n, n, dtype=torch.float64, device="cuda")
c.addmm_(a, a.t(), alpha=-1.0)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(5):
    c.addmm_(a, a.t(), alpha=-1.0)
e.record()
torch.cuda.synchronize()
t = s.elapsed_time(e) / 5 / 1e3
print(f"vendor dgemm {n}x{n}x{k} (NT, beta=1): {t*1e3:9.2f} ms  {2*n*n*k/t/1e12:6.2f} TF/s", flush=True)
