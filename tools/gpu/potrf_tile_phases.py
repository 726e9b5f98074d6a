"""Phase ablation of the single-workgroup tile Cholesky (dpl_debug_set_phase_mask):
bit 1 = stage next Y in LDS, 2 = left-looking block products, 4 = 16x16 factor+inverse,
8 = apply inv(D)^H and store.  Timings only (skipped phases leave wrong numbers)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

from dplasma_amd.constants import dplasmaLower  # noqa: E402
from dplasma_amd.ops import _lib  # noqa: E402
from dplasma_amd.ops import tile_ops as ops  # noqa: E402


def main():
    lib = _lib.load()
    for n in (256, 512):
        lda = 8192
        M = torch.randn(n, n, dtype=torch.float64, device="cuda")
        S = M @ M.T + n * torch.eye(n, dtype=torch.float64, device="cuda")
        buf = torch.zeros(lda * n, dtype=torch.float64, device="cuda")
        view = torch.as_strided(buf, (n, n), (1, lda), 0)
        info = torch.zeros(1, dtype=torch.int32, device="cuda")
        for mask in (0xff, 0xff & ~1, 0xff & ~2, 0xff & ~4, 0xff & ~8, 0):
            lib.dpl_debug_set_phase_mask(mask)
            ts = []
            for rep in range(8):
                view.copy_(S)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ops.potrf_tile(dplasmaLower, buf, 0, n, lda, info, 0)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            ts = sorted(ts[2:])
            print(f"n={n} mask={mask:#04x}: median {ts[len(ts) // 2]:8.1f} us", flush=True)
        lib.dpl_debug_set_phase_mask(0xff)


if __name__ == "__main__":
    main()
