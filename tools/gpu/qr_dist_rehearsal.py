"""Multi-rank rehearsal of the 1 x Q stacked-domain QR on GPU ranks (gloo moves the tensors through
the host when ranks share a device):

  DPLASMA_DIST_BACKEND=gloo python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
      tools/gpu/qr_dist_rehearsal.py [N] [NB]

Factors A = QR on a 1 x world grid, forms Q (ungqr) and checks ||Q^T Q - I|| and ||QR - A|| / ||A||."""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    NB = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dist.init_process_group(os.environ.get("DPLASMA_DIST_BACKEND", "gloo"))
    import dplasma_amd as dp
    from dplasma_amd.models import qr_panel
    ctx = dp.init(P=1)
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plrnt(ctx, A, 3872)
    a = A.to_dense_local().cpu()
    T = dp.block_cyclic(ctx, torch.float64, 32, NB, A.mt * 32, N)
    assert qr_panel.usable(A, dp.models.qrtree.FlatTree(A.mt, A.nt))
    dp.geqrf(ctx, A, T)
    Q = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.ungqr(ctx, A, T, Q)
    torch.cuda.synchronize()
    full = [A.to_dense_local().cpu(), Q.to_dense_local().cpu(), a]
    for t in full:
        dist.all_reduce(t)
    r, q, a0 = torch.triu(full[0]), full[1], full[2]
    orth = (q.T @ q - torch.eye(N, dtype=torch.float64)).abs().max().item()
    res = (q @ r - a0).abs().max().item() / a0.abs().max().item()
    ok = orth < 1e-12 * N and res < 1e-12 * N
    if ctx.rank == 0:
        print(f"qr 1x{ctx.world} N={N} NB={NB}: orth {orth:.3e} residual {res:.3e} : {'SUCCESS' if ok else 'FAIL'}",
              flush=True)
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
