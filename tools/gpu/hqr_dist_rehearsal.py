"""Multi-rank rehearsal of the P x Q stacked-domain HQR (geqrf_param / ungqr_param / geqrs_param) on
GPU ranks; gloo moves tensors through the host when ranks share one device:

  DPLASMA_DIST_BACKEND=gloo python -m torch.distributed.run --nproc-per-node 4 --master-addr 127.0.0.1 \\
      tools/gpu/hqr_dist_rehearsal.py [N] [NB] [P]

Checks ||Q^T Q - I||, ||QR - A|| / ||A|| against the reference's tolerance style and reports the time
of the factorisation (meaningless as performance under gloo)."""
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    NB = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    P = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dist.init_process_group(os.environ.get("DPLASMA_DIST_BACKEND", "gloo"))
    import dplasma_amd as dp
    from dplasma_amd.models import qr_panel
    ctx = dp.init(P=P)
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plrnt(ctx, A, 3872)
    a = A.to_dense_local().cpu()
    IB = 32
    TS = dp.block_cyclic(ctx, torch.float64, IB, NB, A.mt * IB, N)
    TT = dp.block_cyclic(ctx, torch.float64, IB, NB, A.mt * IB, N)
    tree = dp.hqr_init(dp.dplasmaNoTrans, A, dp.dplasma_FLAT_TREE, dp.dplasma_FLAT_TREE, A.mt, P)
    assert qr_panel.usable(A, tree)
    tp = dp.geqrf_param_New(ctx, tree, A, TS, TT)
    ctx.barrier()
    t0 = time.perf_counter()
    tp.execute(ctx)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    Q = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.ungqr_param(ctx, tree, A, TS, TT, Q)
    torch.cuda.synchronize()
    full = [A.to_dense_local().cpu(), Q.to_dense_local().cpu(), a]
    for x in full:
        dist.all_reduce(x)
    r, q, a0 = torch.triu(full[0]), full[1], full[2]
    orth = (q.T @ q - torch.eye(N, dtype=torch.float64)).abs().max().item()
    res = (q @ r - a0).abs().max().item() / a0.abs().max().item()
    ok = orth < 1e-12 * N and res < 1e-12 * N
    if ctx.rank == 0:
        print(f"hqr {ctx.P}x{ctx.Q} N={N} NB={NB}: {t:.3f} s, orth {orth:.3e} residual {res:.3e} : "
              f"{'SUCCESS' if ok else 'FAIL'}", flush=True)
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
