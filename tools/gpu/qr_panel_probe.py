"""Time the persistent QR panel kernel on TS-like (dense) and TT-like (two stacked upper triangles) panels and
report workgroup 0's phase timers / fast-vs-exact column counts (dpl_qr_panel_set_prof).

python tools/gpu/qr_panel_probe.py [--nb 256]"""
import argparse
import ctypes

import torch

from dplasma_amd.ops import _lib, tile_ops as ops

PH = ["col-step", "col-barrier", "exact-reduce", "Y-partials", "Y-reduce+Tb", "trailing", "T-coupling", "load"]


def run(M, nb, tt, reps=5):
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    if tt == "real":
        h = M // 2
        P0 = torch.zeros(M, nb, dtype=torch.float64, device=dev)
        P0[:h] = torch.linalg.qr(torch.randn(16384, nb, dtype=torch.float64, device=dev), mode="r")[1]
        P0[h:] = torch.linalg.qr(torch.randn(16384, nb, dtype=torch.float64, device=dev), mode="r")[1]
    elif tt:
        h = M // 2
        P0 = torch.zeros(M, nb, dtype=torch.float64, device=dev)
        P0[:h] = torch.triu(torch.randn(h, nb, dtype=torch.float64, device=dev))
        P0[h:] = torch.triu(torch.randn(M - h, nb, dtype=torch.float64, device=dev))
    else:
        P0 = torch.randn(M, nb, dtype=torch.float64, device=dev)
    ld = M
    V = torch.zeros(ld * nb, dtype=torch.float64, device=dev)
    Tm = torch.zeros(nb * nb, dtype=torch.float64, device=dev)
    ws = ops.qr_panel_workspace(nb, nb, torch.float64, dev)
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    prof = torch.zeros(16, dtype=torch.int64, device=dev)
    lib = _lib.load()
    ts = []
    for r in range(reps + 1):
        P = P0.t().contiguous().view(-1).clone()     # column-major
        if r == reps:
            lib.dpl_qr_panel_set_prof(ctypes.c_void_p(prof.data_ptr()))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.qr_panel(P, ld, M, nb, nb, V, ld, Tm, nb, ws, info)
        e1.record()
        torch.cuda.synchronize()
        if r == reps:
            lib.dpl_qr_panel_set_prof(ctypes.c_void_p(0))
        elif r > 0:
            ts.append(e0.elapsed_time(e1))
    R = torch.triu(P.view(nb, M).t()[:nb])
    ref = torch.linalg.qr(P0, mode="r")[1]
    err = (R.abs() - ref.abs()).abs().max().item() / ref.abs().max().item()
    # Q R with Q = I - V T V^T from the kernel's explicit V and T: the factorisation itself, not only |R|
    Vm = V.view(nb, ld).t()[:M]
    Tt = torch.triu(Tm.view(nb, nb).t())
    X = torch.zeros(M, nb, dtype=torch.float64, device=dev)
    X[:nb] = R
    rec = X - Vm @ (Tt @ (Vm.t() @ X))
    qerr = ((rec - P0).abs().max() / P0.abs().max()).item()
    p = prof.cpu().tolist()
    tot = sum(p[:8]) or 1
    phases = ", ".join(f"{PH[i]} {p[i] / 100:.0f}us" for i in range(8) if p[i])
    if p[13]:
        phases += f", (col-effects {p[13] / 100:.0f}us)"
    import os
    gm = int(os.environ.get("DPLASMA_QP_GMIN", "0"))
    rm = int(os.environ.get("DPLASMA_QP_RMAX", "0"))
    gq = max(-(-M // 256), min(gm, M), -(-M // rm) if rm else 0)
    print(f"M={M:6d} {('TTr' if tt == 'real' else 'TT') if tt else 'TS'} G={min(gq, 256):3d}  {min(ts):7.3f} ms  fast {p[8]} exact {p[9]} "
          f"first_exact {p[10]}  |R| err {err:.1e}  QR err {qerr:.1e}\n    {phases}", flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--nb", type=int, default=256)
    a = ap.parse_args()
    for M, tt in [(256, False), (512, False), (512, True), (512, "real"), (1024, True), (4096, False), (32768, False)]:
        run(M, a.nb, tt)
