"""Phase timeline of the dataflow diagonal-tile Cholesky (potrf_rb.hip) from its in-kernel
s_memrealtime stamps (100 MHz): per step k, the Z_k hand-off to WG k+1 and WG k+1's TRSM / SYRK /
factorisation, i.e. the kernel's critical path.  Alone, beside an 8192^3 GEMM, and beside the GEMM
restricted to all CUs but R (R = 16, 32: 2 / 4 per XCD) with the tile kernel on the R reserved CUs.

  python tools/gpu/potrf_rb_trace.py [n] [R ...]
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

from dplasma_amd.constants import dplasmaLower, dplasmaNoTrans  # noqa: E402
from dplasma_amd.ops import _lib  # noqa: E402
from dplasma_amd.ops import tile_ops as ops  # noqa: E402
from dplasma_amd.ops.batch import GemmBatch  # noqa: E402
from dplasma_amd.context import Context  # noqa: E402


def show(tr, nblk, tag):
    t = tr.view(-1, 64).double() / 100.0  # us
    t0 = t[:nblk, 0].min()
    t = t - t0
    print(f"--- {tag}: WG start spread {float(t[:nblk, 0].max()):.1f} us, end {float(t[nblk - 1, 51]):.1f} us")
    print(" k | Z_k pub | WG k+1 poll-> TRSM done -> upd done | diag start chol done pub | hop  trsm  upd  chol  pub")
    for k in range(nblk - 1):
        zp = float(t[k, 51])
        i = k + 1
        p, tr_, up = float(t[i, 1 + 3 * k]), float(t[i, 2 + 3 * k]), float(t[i, 3 + 3 * k])
        ds, dc, dp = float(t[i, 49]), float(t[i, 50]), float(t[i, 51])
        print(f"{k:2d} | {zp:7.1f} | {p:7.1f} {tr_:7.1f} {up:7.1f} | {ds:7.1f} {dc:7.1f} {dp:7.1f} |"
              f" {p - zp:4.1f} {tr_ - p:5.1f} {up - tr_:4.1f} {dc - ds:5.1f} {dp - dc:4.1f}")
    last = nblk - 1
    print("last WG per-step (poll, trsm, upd):",
          " ".join(f"{float(t[last, 1 + 3 * k]):.0f}/{float(t[last, 2 + 3 * k] - t[last, 1 + 3 * k]):.1f}/"
                   f"{float(t[last, 3 + 3 * k] - t[last, 2 + 3 * k]):.1f}" for k in range(last)))


def masked(lib, ncu, cus):
    import ctypes
    nw = (ncu + 31) // 32
    words = [0] * nw
    for c in cus:
        words[c // 32] |= 1 << (c % 32)
    arr = (ctypes.c_uint * nw)(*words)
    out = ctypes.c_void_p()
    _lib.check(lib.dpl_stream_cumask(ctypes.cast(arr, ctypes.c_void_p), nw, ctypes.byref(out)), "stream_cumask")
    return torch.cuda.ExternalStream(out.value)


def main():
    lib = _lib.load()
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    nblk = (n + 31) // 32
    lda = n
    M = torch.randn(n, n, dtype=torch.float64, device="cuda")
    S = M @ M.T + n * torch.eye(n, dtype=torch.float64, device="cuda")
    buf = torch.zeros(lda * n, dtype=torch.float64, device="cuda")
    view = torch.as_strided(buf, (n, n), (1, lda), 0)
    info = torch.zeros(1, dtype=torch.int32, device="cuda")
    tr = torch.zeros(64 * nblk, dtype=torch.int64, device="cuda")
    N = 8192
    big = torch.randn(3 * N * N, dtype=torch.float64, device="cuda")
    gb = GemmBatch()
    for i in range(0, N, 512):
        for j in range(0, N, 512):
            gb.add(2 * N * N + i + j * N, 512, 512, [(i, N * N + j * N, N)], 0)
    gb.finalize()
    lo = torch.cuda.Stream(priority=0)
    hi = torch.cuda.Stream(priority=-1)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    modes = [(False, None, None, "alone"), (True, lo, hi, "beside GEMM")]
    for R in [int(a) for a in sys.argv[2:]] or [16, 32]:
        keep = Context.reserve_mask(ncu, R)
        rsv = [c for c in range(ncu) if c not in set(keep)]
        modes.append((True, masked(lib, ncu, keep), masked(lib, ncu, rsv),
                      f"beside GEMM on {len(keep)} CUs, tile on the other {len(rsv)}"))
        modes.append((True, masked(lib, ncu, keep), hi, f"beside GEMM on {len(keep)} CUs, tile unmasked"))
    for beside, lo, hi, tag in modes:
        for rep in range(4):
            view.copy_(S)
            torch.cuda.synchronize()
            if beside:
                with torch.cuda.stream(lo):
                    ops.gemm(dplasmaNoTrans, dplasmaNoTrans, 1.0, big, N, big, N, 0.0, big, N, gb)
            with torch.cuda.stream(hi):
                if beside:
                    torch.cuda._sleep(20000)
                lib.dpl_potrf_rb_set_trace(tr.data_ptr() if rep == 3 else None)
                ops.potrf_tile(dplasmaLower, buf, 0, n, lda, info, 0)
                lib.dpl_potrf_rb_set_trace(None)
            torch.cuda.synchronize()
        show(tr.cpu(), nblk, tag)


if __name__ == "__main__":
    main()
