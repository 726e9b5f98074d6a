"""Phase timers of the persistent QR panel kernel (workgroup 0) for a few panel heights.

python tools/gpu/qr_panel_prof.py [M ...]   (nc = kf = 256, fp64)"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

from dplasma_amd.ops import _lib  # noqa: E402
from dplasma_amd.ops import tile_ops as ops  # noqa: E402

NAMES = ["block Gram", "column steps", "exact columns", "Y partials", "Y barriers+sum", "trailing upd", "T coupling",
         "block load"]


def main():
    dev = torch.device("cuda:0")
    lib = _lib.load()
    prof = torch.zeros(16, dtype=torch.int64, device=dev)
    nc = kf = 256
    for M in [int(x) for x in sys.argv[1:]] or [256, 1024, 4096, 16384, 65536]:
        ld = M
        P = torch.randn(ld * nc, dtype=torch.float64, device=dev)
        V = torch.zeros(ld * kf, dtype=torch.float64, device=dev)
        Tm = torch.zeros(kf * kf, dtype=torch.float64, device=dev)
        ws = ops.qr_panel_workspace(nc, kf, torch.float64, dev)
        info = torch.zeros(1, dtype=torch.int32, device=dev)
        ops.qr_panel(P, ld, M, nc, kf, V, ld, Tm, kf, ws, info)   # warm-up
        torch.cuda.synchronize()
        P.copy_(torch.randn(ld * nc, dtype=torch.float64, device=dev))   # fresh data (not the factored panel)
        prof.zero_()
        lib.dpl_qr_panel_set_prof(prof.data_ptr())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.qr_panel(P, ld, M, nc, kf, V, ld, Tm, kf, ws, info)
        e1.record()
        torch.cuda.synchronize()
        lib.dpl_qr_panel_set_prof(None)
        t_all = prof.cpu()
        t = t_all[:8].tolist()
        import struct
        f2 = lambda v: struct.unpack("d", struct.pack("q", int(v)))[0]  # noqa: E731
        print(f"   fast columns {int(t_all[8])}  exact columns {int(t_all[9])}  first exact j={int(t_all[10])} "
              f"x2={f2(t_all[11]):.4g} g0={f2(t_all[12]):.4g}")
        tot = sum(t)
        print(f"M={M:6d} wall {e0.elapsed_time(e1):7.3f} ms  info={int(info.item())}  " +
              "  ".join(f"{n}: {v / 1e5:.3f} ms" for n, v in zip(NAMES, t)) + f"  (sum {tot / 1e5:.3f} ms)",
              flush=True)


if __name__ == "__main__":
    main()
