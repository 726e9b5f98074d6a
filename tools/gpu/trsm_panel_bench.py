"""POTRF panel TRSM in isolation: inverse + copy + MFMA GEMM (ops.trsm) vs the register-resident
row-block kernel (ops.trsm_rb), for a panel of `ntiles` 512 x 512 tiles below a factored tile.

  python tools/gpu/trsm_panel_bench.py [ntiles ...]
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

from dplasma_amd.constants import dplasmaConjTrans, dplasmaLower, dplasmaNonUnit, dplasmaRight  # noqa: E402
from dplasma_amd.ops import _lib  # noqa: E402
from dplasma_amd.ops import tile_ops as ops  # noqa: E402
from dplasma_amd.ops.batch import TileBatch  # noqa: E402


def timeit(fn, reps=8):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts = sorted(ts[2:])
    return ts[len(ts) // 2]


def main():
    _lib.load()
    n = 512
    for nt in [int(a) for a in sys.argv[1:]] or [15, 63, 127]:
        M = n * (nt + 1)
        ld = M
        A = torch.randn(ld * n, dtype=torch.float64, device="cuda")
        T = torch.randn(n, n, dtype=torch.float64, device="cuda")
        S = T @ T.T + n * torch.eye(n, dtype=torch.float64, device="cuda")
        torch.as_strided(A, (n, n), (1, ld), 0).copy_(S)
        info = torch.zeros(1, dtype=torch.int32, device="cuda")
        zbuf = torch.empty(ops.rb_zbuf_size(), dtype=torch.float64, device="cuda")
        ops.potrf_tile(dplasmaLower, A, 0, n, ld, info, 0, zbuf=zbuf)
        tb = TileBatch()
        for i in range(1, nt + 1):
            tb.add(0, n, n, b_off=i * n)
        tb.finalize()
        panel = ops.RbPanel(dplasmaLower, [(i * n, n) for i in range(1, nt + 1)], ld)
        t_old = timeit(lambda: ops.trsm(dplasmaRight, dplasmaLower, dplasmaConjTrans, dplasmaNonUnit, 1.0, A, ld,
                                        A, ld, tb))
        t_rb = timeit(lambda: ops.trsm_rb(dplasmaLower, n, A, 0, ld, zbuf, panel, A, ld))
        t_prep = timeit(lambda: ops.trsm_rb_prep(dplasmaLower, n, A, 0, ld, zbuf))
        fl = float(nt) * n * n * n
        print(f"panel {nt:4d} tiles: inverse+GEMM {t_old:8.1f} us ({fl / t_old / 1e6:6.2f} TF/s)   "
              f"trsm_rb {t_rb:8.1f} us ({fl / t_rb / 1e6:6.2f} TF/s)   prep {t_prep:6.1f} us", flush=True)


if __name__ == "__main__":
    main()
