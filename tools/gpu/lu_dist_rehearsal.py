"""Rehearsal of the distributed-pivoting LU panel (DPLASMA_LU_PANEL=dist, ops.lu_dist_ops) with ranks
sharing ONE GPU: the per-column candidate exchange runs through IPC-mapped exchange buffers between
the processes exactly as between GPUs of a node (gloo only carries the host-side setup, the diagonal
tile replica and the trailing row moves):

  DPLASMA_DIST_BACKEND=gloo python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
      tools/gpu/lu_dist_rehearsal.py [N] [NB] [P]      (P < world: a P x world/P grid)

Checks: the exchange is device-side (``ipc``), pivots are identical to the one-process factorisation
of the same matrix on the same GPU, and the factors agree.  Prints the factorisation time and the mean
duration per panel column of the exchange kernel (CUDA events around every block launch of one
panel -- ranks share the GPU, so this is an upper bound of the per-GPU figure)."""
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    NB = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    P = int(sys.argv[3]) if len(sys.argv) > 3 else int(os.environ.get("WORLD_SIZE", "2"))
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dist.init_process_group(os.environ.get("DPLASMA_DIST_BACKEND", "gloo"))
    os.environ.setdefault("DPLASMA_LU_PANEL", "dist")
    import dplasma_amd as dp
    from dplasma_amd.models.lu import _gather_ipiv
    from dplasma_amd.ops import lu_dist_ops
    ctx = dp.init(P=P)
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plrnt(ctx, A, 3872)
    IPIV = dp.ptgpanel_ipiv_descriptor(ctx, A)
    tp = dp.getrf_ptgpanel_New(ctx, A, IPIV)
    st = tp._state
    mode = "ipc" if (st.xc is not None and st.xc.ok) else "host"
    # per-column exchange cost: time every dist block launch of the first panel this rank factors
    times = []
    orig = lu_dist_ops.DistPanelLU.run

    def timed(self, *a, **kw):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        # no host synchronisation inside the panel: torch raises on any synchronizing call
        # (.item(), .cpu(), blocking copies) while the panel's kernels are issued
        torch.cuda.set_sync_debug_mode("error" if mode == "ipc" else "default")
        try:
            orig(self, *a, **kw)
        finally:
            torch.cuda.set_sync_debug_mode("default")
        e1.record()
        times.append((e0, e1, self.kf))
    lu_dist_ops.DistPanelLU.run = timed
    ctx.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    info = tp.execute(ctx)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    lu_dist_ops.DistPanelLU.run = orig
    piv = _gather_ipiv(ctx, IPIV)
    fac = A.to_dense_local().cpu()
    dist.all_reduce(fac)
    panel_ms = [a.elapsed_time(b) for a, b, _ in times]
    ncol = sum(k for _, _, k in times)
    tp.destruct()
    # one process, same matrix, same GPU
    lctx = ctx.local()
    B = dp.block_cyclic(lctx, torch.float64, NB, NB, N, N)
    dp.plrnt(lctx, B, 3872)
    IP1 = dp.ipiv_descriptor(lctx, B)
    info1 = dp.getrf_1d(lctx, B, IP1)
    piv1 = _gather_ipiv(lctx, IP1)
    same = bool(np.array_equal(piv, piv1))
    diff = (fac - B.to_dense_local().cpu()).abs().max().item()
    # the device exchange is required of the distributed-pivoting panel only (gather-mode panels -- factored whole
    # by the ranks that need them, DPLASMA_LU_PANEL=gather -- have no per-column exchange)
    need_ipc = os.environ.get("DPLASMA_LU_PANEL") == "dist" and os.environ.get("DPLASMA_LU_XCHG") != "host"
    ok = info == 0 and info1 == 0 and same and diff < 1e-8 and (mode == "ipc" or not need_ipc)
    if not ok and ctx.rank == 0:   # which tiles differ (tile row, tile column, max |diff|), first ones
        dd = (fac - B.to_dense_local().cpu()).abs()
        bad = [(m, n, dd[m * NB:(m + 1) * NB, n * NB:(n + 1) * NB].max().item())
               for m in range(-(-N // NB)) for n in range(-(-N // NB))]
        bad = [b for b in bad if b[2] > 1e-8]
        print(f"rank 0: {len(bad)} tiles differ; first: {bad[:24]}", flush=True)
    flags = torch.tensor([int(ok)])
    dist.all_reduce(flags, op=dist.ReduceOp.MIN)
    print(f"rank {ctx.rank}: lu dist {ctx.P}x{ctx.Q} N={N} NB={NB} exchange={mode}: {t:.3f} s, panels on this rank "
          f"{len(panel_ms)} ({sum(panel_ms):.2f} ms, {1e3 * sum(panel_ms) / max(1, ncol):.2f} us per column), "
          f"no host sync inside a panel: {mode == 'ipc'}, "
          f"pivots identical to one process: {same}, max |factor diff| {diff:.2e} : "
          f"{'SUCCESS' if ok else 'FAIL'}", flush=True)
    from dplasma_amd.ops import lu_dist_ops
    lu_dist_ops.release_all()   # IPC mappings closed before the runtime's teardown (see lu_dist_ops._at_exit)
    dist.destroy_process_group()
    sys.exit(0 if int(flags[0]) == 1 else 1)


if __name__ == "__main__":
    main()
