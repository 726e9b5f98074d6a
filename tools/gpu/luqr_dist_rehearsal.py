"""Rehearsal of the device-decided hybrid LU-QR on several processes (models/lu_qr.py _run_devcrit_dist) with
ranks sharing ONE GPU (gloo carries the collectives; on a node of GPUs they are RCCL):

  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/gpu/luqr_dist_rehearsal.py \\
      [N] [NB] [P]

For each data-dependent criterion: the device-decided run (both branches issued under the device flag) against the
host-decided one (DPLASMA_LUQR_DEVCRIT=0) on the same matrix: same lu_tab, same pivots, factors equal to rounding,
and the solve residual of trsmpl_qrf + trsm(U)."""
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def run(ctx, dp, lu_qr, qrtree, N, NB, ib, crit, alpha, devcrit):
    os.environ["DPLASMA_LUQR_DEVCRIT"] = "1" if devcrit else "0"
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plrnt(ctx, A, 7)
    A0 = A.to_dense_local()
    TS = dp.block_cyclic(ctx, torch.float64, ib, NB, A.mt * ib, N)
    TT = dp.block_cyclic(ctx, torch.float64, ib, NB, A.mt * ib, N)
    IP = dp.qrf_ipiv_descriptor(ctx, A)
    tree = qrtree.hqr_init(dp.dplasmaNoTrans, A, qrtree.GREEDY_TREE, qrtree.FLAT_TREE, 2, None)
    tp = lu_qr.getrf_qrf_New(ctx, tree, A, IP, TS, TT, crit, alpha)
    ctx.sync()
    ctx.barrier()
    t0 = time.perf_counter()
    tp.execute(ctx)
    ctx.sync()
    el = time.perf_counter() - t0
    x = A.to_dense_local()
    dist.all_reduce(x)
    ip = IP.to_dense_local()
    dist.all_reduce(ip)
    dist.all_reduce(A0)
    return tp, list(tp.lu_tab), x, ip, el, A0


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    NB = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    P = int(sys.argv[3]) if len(sys.argv) > 3 else int(os.environ.get("WORLD_SIZE", "2"))
    gpu = torch.cuda.is_available()
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    if gpu:
        torch.cuda.set_device(local)
    dist.init_process_group("gloo")
    import dplasma_amd as dp
    from dplasma_amd.models import lu_qr, qrtree
    ctx = dp.init(P=P, device=f"cuda:{local}" if gpu else "cpu")
    me = dist.get_rank()
    ok_all = True
    for crit, alpha in ((dp.HIGHAM_CRITERIUM, 0.02), (dp.HIGHAM_SUM_CRITERIUM, 1.0), (dp.HIGHAM_MAX_CRITERIUM, 2.0),
                        (dp.HIGHAM_MOY_CRITERIUM, 4.0), (dp.MUMPS_CRITERIUM, 1.0), (dp.MUMPS_CRITERIUM, 3.0)):
        tpd, tab_d, xd, ipd, td, A0 = run(ctx, dp, lu_qr, qrtree, N, NB, 32, crit, alpha, True)
        tph, tab_h, xh, iph, th, _ = run(ctx, dp, lu_qr, qrtree, N, NB, 32, crit, alpha, False)
        diff = float((xd - xh).abs().max() / xh.abs().max())
        same = tab_d == tab_h and bool((ipd == iph).all()) and diff < 1e-10 and tpd.devcrit_dist
        ok_all &= same
        if me == 0:
            print(f"crit={crit} alpha={alpha}: devcrit_dist={tpd.devcrit_dist} lu_tab dev {tab_d} host {tab_h} "
                  f"pivots equal {bool((ipd == iph).all())} factor rel diff {diff:.2e}  time dev {td * 1e3:.1f} ms "
                  f"host {th * 1e3:.1f} ms -> {'OK' if same else 'MISMATCH'}", flush=True)
    ok = torch.tensor([1.0 if ok_all else 0.0])
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if me == 0:
        print("LUQR_DIST_REHEARSAL", "PASS" if ok.item() > 0 else "FAIL", flush=True)
    dist.destroy_process_group()
    sys.exit(0 if ok.item() > 0 else 1)


if __name__ == "__main__":
    main()
