"""Diagonal-tile Cholesky kernels in isolation: single-workgroup left-looking kernel vs the
128-wide blocked composition (POTRF + TRSM + masked GEMM launches).

  python tools/gpu/potrf_tile_bench.py [NB ...]
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

from dplasma_amd.constants import dplasmaLower  # noqa: E402
from dplasma_amd.ops import _lib  # noqa: E402
from dplasma_amd.ops import tile_ops as ops  # noqa: E402


def main():
    _lib.load()
    sizes = [int(a) for a in sys.argv[1:]] or [256, 512, 1024]
    for n in sizes:
        lda = 8192
        M = torch.randn(n, n, dtype=torch.float64, device="cuda")
        S = M @ M.T + n * torch.eye(n, dtype=torch.float64, device="cuda")
        buf = torch.zeros(lda * n, dtype=torch.float64, device="cuda")
        view = torch.as_strided(buf, (n, n), (1, lda), 0)
        info = torch.zeros(1, dtype=torch.int32, device="cuda")
        L = torch.linalg.cholesky(S)
        for name, fn in (("single", ops.potrf_tile), ("blocked128", ops.potrf_tile_blocked),
                         ("blocked64", lambda *a: ops.potrf_tile_blocked(*a, nb=64))):
            if name == "single" and n > 512:
                continue
            ts = []
            for rep in range(12):
                view.copy_(S)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn(dplasmaLower, buf, 0, n, lda, info, 0)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            err = (view.tril() - L).abs().max().item()
            ts = sorted(ts[2:])
            print(f"potrf tile n={n:5d} {name:11s}: median {ts[len(ts) // 2]:8.1f} us  min {ts[0]:8.1f} us"
                  f"  max|L-L_ref| {err:.2e} info {int(info.item())}", flush=True)


if __name__ == "__main__":
    main()
