"""Rehearsal of the distributed device task runtime Cholesky (models/potrf_dtr_dist.py, process mode)
with the ranks of a P x Q grid sharing ONE GPU: every rank runs its own persistent launch (capped to
its share of the workgroups, DPLASMA_DTR_WG), SEND tasks store strips into the peers' IPC-mapped
receive buffers with system-scope stores and bump their IPC-mapped counters -- exactly the mechanism
between GPUs of a node; gloo carries only the host-side setup (handles, barriers, info).

  DPLASMA_DIST_BACKEND=gloo python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
      tools/gpu/dtr_dist_rehearsal.py [N] [P] [runs]

Checks the assembled factor (every rank's tiles gathered on rank 0) against the pristine matrix with the
reference residual test, and prints each run's time."""
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    runs = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    torch.cuda.set_device(0)
    dist.init_process_group(os.environ.get("DPLASMA_DIST_BACKEND", "gloo"))
    world = dist.get_world_size()
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    # the ranks share the GPU: each launch gets its share of the 2 x #CUs resident workgroups
    os.environ.setdefault("DPLASMA_DTR_WG", str(max(64, ncu // world)))
    os.environ["DPLASMA_POTRF_ENGINE"] = "dtr"
    import dplasma_amd as dp
    ctx = dp.init(P=P)
    A = dp.block_cyclic(ctx, torch.float64, 512, 512, N, N)
    dp.plghe(ctx, float(N), dp.dplasmaLower, A, 3872)
    A0 = A.data.clone()
    tp = dp.potrf_New(ctx, dp.dplasmaLower, A)
    kind = "dtr-dist" if getattr(tp, "dtr_plan", None) is not None else "other engine"
    B = dp.block_cyclic(ctx, torch.float64, 512, 512, N, N)
    B.data.copy_(A0)
    M = B.to_dense_local().cpu()
    dist.all_reduce(M)
    Ms = torch.tril(M)
    Ms = Ms + torch.tril(Ms, -1).T
    Lref = torch.linalg.cholesky(Ms.cuda()).cpu() if ctx.rank == 0 else None
    nt = N // 512
    fails = 0
    for rep in range(runs):
        A.data.copy_(A0)
        torch.cuda.synchronize()
        ctx.barrier()
        t0 = time.perf_counter()
        info = tp.execute(ctx)
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        L = A.to_dense_local().cpu()
        dist.all_reduce(L)
        if ctx.rank == 0:
            Lt = torch.tril(L)
            r = (Lt @ Lt.T - Ms).abs().max().item() / (Ms.abs().max().item() * N * 2.22e-16)
            ok = r < 60
            fails += not ok
            msg = ""
            if not ok:
                # the tiles of L that differ from the one-process factor, in factorisation order
                bad = []
                for j in range(nt):
                    for i in range(j, nt):
                        d = (Lt[i * 512:(i + 1) * 512, j * 512:(j + 1) * 512] -
                             Lref[i * 512:(i + 1) * 512, j * 512:(j + 1) * 512]).abs().max().item()
                        if d > 1e-8:
                            bad.append((j, i, d))
                msg = f" bad tiles {len(bad)} first (k, i, err): {bad[:6]}"
            print(f"run {rep}: {t * 1e3:.1f} ms info={info} ({kind}) residual {r:.3e} "
                  f"{'ok' if ok else 'WRONG'}{msg}", flush=True)
    if ctx.rank == 0:
        print(f"[****] DTR-DIST rehearsal world={world} grid={P}x{world // P} N={N}: {runs - fails}/{runs} runs correct "
              f"{'SUCCESS' if fails == 0 else 'FAILED'}", flush=True)
    from dplasma_amd.models import potrf_dtr_dist
    potrf_dtr_dist.release_all()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
