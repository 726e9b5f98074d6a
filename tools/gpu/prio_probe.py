"""Why is the panel chain slow beside the bulk trailing update?  Dispatch probe.

A bulk GEMM shaped like a Cholesky trailing update (lower tiles of an nt x nt tile matrix, k-run of
`kp` panels) runs on a low-priority stream; the panel chain (tile POTRF + register-resident panel
TRSM of `nt` tiles) is launched right behind it on a high-priority stream.  The panel's latency
(host launch -> TRSM end, device events) is measured with the bulk GEMM

  * uncapped (one workgroup per 128x128 sub-tile: ~nt^2/2 * 16 pending workgroups),
  * capped to `cap` resident workgroups that walk the sub-tiles grid-stride (k_gemm_full<PERSIST>),

so a cap of 2 x #CUs (the GEMM's full occupancy) separates "the SIMDs are busy" from "the
dispatcher is clogged with the GEMM's pending workgroups".

  python tools/gpu/prio_probe.py [nt] [kp] [caps...]
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

from dplasma_amd.constants import dplasmaLower, dplasmaNoTrans, dplasmaConjTrans  # noqa: E402
from dplasma_amd.ops import _lib  # noqa: E402
from dplasma_amd.ops import tile_ops as ops  # noqa: E402
from dplasma_amd.ops.batch import GemmBatch, MASK_LOWER  # noqa: E402


def main():
    _lib.load()
    nt = int(sys.argv[1]) if len(sys.argv) > 1 else 96
    kp = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    caps = [int(a) for a in sys.argv[3:]] or [0, 512, 768, 1024]
    n = 512
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    N = nt * n
    C = torch.zeros(N * N, dtype=torch.float64, device="cuda")
    W = torch.randn(N * kp * n, dtype=torch.float64, device="cuda") * 1e-3   # panel slab: N x (kp*n), ld N
    gb = GemmBatch()
    for j in range(nt):
        for i in range(j, nt):
            gb.add(i * n + j * n * N, n, n, [(i * n + q * n * N, j * n + q * n * N, n) for q in range(kp)],
                   MASK_LOWER if i == j else 0)
    gb.finalize()
    flops = 2.0 * gb.flops_mnk
    # panel: a separate N x n column block, SPD tile on top
    P = torch.randn(N * n, dtype=torch.float64, device="cuda")
    T = torch.randn(n, n, dtype=torch.float64, device="cuda")
    S = T @ T.T + n * torch.eye(n, dtype=torch.float64, device="cuda")
    P0 = P.clone()
    torch.as_strided(P0, (n, n), (1, N), 0).copy_(S)
    info = torch.zeros(1, dtype=torch.int32, device="cuda")
    zbuf = torch.empty(ops.rb_zbuf_size(), dtype=torch.float64, device="cuda")
    panel = ops.RbPanel(dplasmaLower, [(i * n, n) for i in range(1, nt)], N)
    lo, hi = torch.cuda.Stream.priority_range()
    s_bulk = torch.cuda.Stream(priority=lo)
    s_pan = torch.cuda.Stream(priority=hi)

    mode = {"what": "both"}
    tiny = torch.zeros(256, device="cuda")

    def run_panel():
        if mode["what"] == "tiny":      # a trivial elementwise kernel: queueing, not resources
            tiny.add_(1.0)
            return
        if mode["what"] in ("both", "potrf"):
            ops.potrf_tile(dplasmaLower, P, 0, n, N, info, 0, zbuf=zbuf)
        if mode["what"] in ("both", "trsm"):
            ops.trsm_rb(dplasmaLower, n, P, 0, N, zbuf, panel, P, N)

    def ev():
        return torch.cuda.Event(enable_timing=True)

    def one(cap, with_panel, with_bulk):
        P.copy_(P0)
        torch.cuda.synchronize()
        e0, eb, ep0, ep = ev(), ev(), ev(), ev()
        cur = torch.cuda.current_stream()
        e0.record(cur)
        if with_bulk:
            s_bulk.wait_stream(cur)
            with torch.cuda.stream(s_bulk):
                with ops.gemm_wg_cap(cap):
                    ops.gemm(dplasmaNoTrans, dplasmaConjTrans, -1.0, W, N, W, N, 1.0, C, N, gb)
                eb.record(s_bulk)
        if with_panel:
            s_pan.wait_stream(cur)
            with torch.cuda.stream(s_pan):
                ep0.record(s_pan)
                run_panel()
                ep.record(s_pan)
        torch.cuda.synchronize()
        tb = e0.elapsed_time(eb) if with_bulk else float("nan")
        tp = ep0.elapsed_time(ep) if with_panel else float("nan")
        return tb, tp

    for _ in range(2):
        one(0, True, True)
    tb0, _ = one(0, False, True)
    _, tp0 = one(0, True, False)
    print(f"# nt={nt} kp={kp} CUs={ncu} bulk items={len(gb.items)}",
          flush=True)
    print(f"bulk alone      : {tb0:9.3f} ms  {flops / tb0 / 1e9:8.2f} TF/s", flush=True)
    print(f"panel alone     : {tp0 * 1e3:9.1f} us", flush=True)
    for what in ("tiny", "potrf", "trsm"):
        mode["what"] = what
        _, ta = one(0, True, False)
        res = [one(0, True, True) for _ in range(3)]
        tp = sorted(r[1] for r in res)[1]
        print(f"panel part {what:6s}: alone {ta * 1e3:9.1f} us, beside the uncapped bulk {tp * 1e3:10.1f} us", flush=True)
    mode["what"] = "both"
    for cap in caps:
        res = [one(cap, True, True) for _ in range(3)]
        tb = sorted(r[0] for r in res)[1]
        tp = sorted(r[1] for r in res)[1]
        tbo, _ = one(cap, False, True)
        print(f"cap {cap:5d}: bulk alone {tbo:9.3f} ms ({flops / tbo / 1e9:6.2f} TF/s) | with panel: bulk {tb:9.3f} ms, "
              f"panel latency {tp * 1e3:10.1f} us", flush=True)


if __name__ == "__main__":
    main()
