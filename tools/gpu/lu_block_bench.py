"""Per-column cost of the persistent pivoting LU block kernel (k_lu_block_persist) vs panel height.

python tools/gpu/lu_block_bench.py [M ...]   (64 columns, fp64; G = ceil(M / 256) workgroups)"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

from dplasma_amd.ops import tile_ops as ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    for M in [int(x) for x in sys.argv[1:]] or [1024, 4096, 8192, 16384, 32768, 65536]:
        bw = 64
        P0 = torch.randn(M * bw, dtype=torch.float64, device=dev)
        P = P0.clone()
        ipiv = torch.zeros(M, dtype=torch.int32, device=dev)
        ws = ops.lu_workspace(M, dev)
        cnt = torch.zeros(4, dtype=torch.int32, device=dev)
        info = torch.zeros(1, dtype=torch.int32, device=dev)
        ts = []
        for r in range(6):
            P.copy_(P0)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.lu_block(P, M, M, 0, bw, ipiv, ws, cnt, info, 0)
            e1.record()
            torch.cuda.synchronize()
            if r:
                ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        # check against torch's LU of the same M x 64 panel (column-major buffer = transposed view)
        LU, piv = torch.linalg.lu_factor(P0.view(bw, M).T)
        same_piv = bool(torch.equal(ipiv[:bw].long() + 1, piv.long()))
        err = float((P.view(bw, M).T - LU).abs().max())
        print(f"M={M:6d} G={-(-M // 256):4d}: {ts[len(ts) // 2]:8.1f} us per 64-column block = "
              f"{ts[len(ts) // 2] / bw:6.2f} us/column  info={int(info.item())} pivots_match={same_piv} "
              f"max|LU-ref|={err:.1e}", flush=True)
        if not same_piv or err > 1e-8 or int(info.item()) != 0:
            bad = (ipiv[:bw].long() + 1 != piv.long()).nonzero()
            print("  first pivot mismatch at column", bad[:4].flatten().tolist(), "ours", ipiv[:8].tolist(),
                  "ref", (piv[:8] - 1).tolist(), "nan", bool(P.isnan().any()), flush=True)
            sys.exit(1)


if __name__ == "__main__":
    main()
