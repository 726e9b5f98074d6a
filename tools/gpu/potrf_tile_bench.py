"""Diagonal-tile Cholesky kernels in isolation and beside a bulk GEMM.

kind 0 = multi-workgroup dataflow kernel (potrf_rb.hip), kind 1 = single-workgroup kernel
(potrf_trsm.hip k_potrf_ll), "blocked128" = 128-wide composition of launches.  "beside GEMM": the
tile runs on a high-priority stream while an 8192^3 MFMA GEMM occupies the chip on another stream
(the situation of the POTRF critical path under the trailing update).

  python tools/gpu/potrf_tile_bench.py [NB ...]
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

from dplasma_amd.constants import dplasmaLower, dplasmaNoTrans  # noqa: E402
from dplasma_amd.ops import _lib  # noqa: E402
from dplasma_amd.ops import tile_ops as ops  # noqa: E402
from dplasma_amd.ops.batch import GemmBatch  # noqa: E402


def kinded(kind):
    def f(*a):
        old = _lib.load().dpl_potrf_tile_set_kind(kind)
        try:
            ops.potrf_tile(*a)
        finally:
            _lib.load().dpl_potrf_tile_set_kind(old)
    return f


def main():
    _lib.load()
    sizes = [int(a) for a in sys.argv[1:]] or [256, 512]
    N = 8192
    big = torch.randn(3 * N * N, dtype=torch.float64, device="cuda")
    gb = GemmBatch()
    for i in range(0, N, 512):
        for j in range(0, N, 512):
            gb.add(2 * N * N + i + j * N, 512, 512, [(i, N * N + j * N, N)], 0)
    gb.finalize()
    lo = torch.cuda.Stream(priority=0)
    hi = torch.cuda.Stream(priority=-1)
    for n in sizes:
        lda = 8192
        M = torch.randn(n, n, dtype=torch.float64, device="cuda")
        S = M @ M.T + n * torch.eye(n, dtype=torch.float64, device="cuda")
        buf = torch.zeros(lda * n, dtype=torch.float64, device="cuda")
        view = torch.as_strided(buf, (n, n), (1, lda), 0)
        info = torch.zeros(1, dtype=torch.int32, device="cuda")
        L = torch.linalg.cholesky(S)
        for name, fn in (("rb", kinded(0)), ("single", kinded(1)), ("blocked128", ops.potrf_tile_blocked)):
            for beside in (False, True):
                ts = []
                for rep in range(12):
                    view.copy_(S)
                    torch.cuda.synchronize()
                    if beside:
                        with torch.cuda.stream(lo):
                            ops.gemm(dplasmaNoTrans, dplasmaNoTrans, 1.0, big, N, big, N, 0.0, big, N, gb)
                    with torch.cuda.stream(hi):
                        if beside:
                            torch.cuda._sleep(20000)  # let the GEMM fill the chip first
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        fn(dplasmaLower, buf, 0, n, lda, info, 0)
                        e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) * 1e3)
                err = (view.tril() - L).abs().max().item()
                ts = sorted(ts[2:])
                tag = "beside GEMM" if beside else "alone      "
                print(f"potrf tile n={n:5d} {name:11s} {tag}: median {ts[len(ts) // 2]:8.1f} us  min {ts[0]:8.1f} us"
                      f"  max|L-L_ref| {err:.2e} info {int(info.item())}", flush=True)


if __name__ == "__main__":
    main()
