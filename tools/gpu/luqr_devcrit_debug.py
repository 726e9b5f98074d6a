"""Step-by-step check of the device-decided LU-QR path (models/lu_qr.py _run_devcrit) against the host path."""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

import dplasma_amd as dp  # noqa: E402
from dplasma_amd.models import lu_qr, qrtree  # noqa: E402
from dplasma_amd.ops import batch as B  # noqa: E402


def build(g, crit, alpha, N, NB, p, dev):
    os.environ["DPLASMA_LUQR_DEVCRIT"] = "1" if dev else "0"
    dt = torch.float64
    A = dp.block_cyclic(g, dt, NB, NB, N, N)
    dp.plrnt(g, A, 7)
    TS = dp.block_cyclic(g, dt, 32, NB, A.mt * 32, N)
    TT = dp.block_cyclic(g, dt, 32, NB, A.mt * 32, N)
    IP = dp.qrf_ipiv_descriptor(g, A)
    tree = qrtree.hqr_init(dp.dplasmaNoTrans, A, qrtree.GREEDY_TREE, qrtree.FLAT_TREE, 2, p)
    tp = dp.getrf_qrf_New(g, tree, A, IP, TS, TT, crit, alpha, [0] * A.mt, p=p)
    return tp, A


def main():
    N, NB, p = int(sys.argv[1]), int(sys.argv[2]), 2
    crit = int(sys.argv[3]) if len(sys.argv) > 3 else dp.HIGHAM_SUM_CRITERIUM
    g = dp.init(device="cuda:0")
    tpd, Ad = build(g, crit, 1.0, N, NB, p, True)
    tph, Ah = build(g, crit, 1.0, N, NB, p, False)
    print("devcrit", tpd.devcrit, tph.devcrit, flush=True)
    for k in range(tpd.minMNT):
        st = lu_qr._Step(Ad, k, p)
        snap = Ad.data.clone()
        buf, view, ipiv, info, colmax = tpd._domain_lu_dev(st)
        flag = tpd._criterion_dev(st, view, info, colmax)
        with B.predicated(flag):
            tpd._lu_step_dev(st, buf, ipiv, flag)
        torch.cuda.synchronize()
        nan1 = bool(torch.isnan(Ad.data).any())
        if int(flag.item()) == 0:
            ch = (Ad.data - snap).abs().max().item()
            print(f"k={k}: skipped LU branch changed A by {ch:.3e}", flush=True)
            if ch > 0:
                for (m, n) in Ad.local_tiles():
                    e = (Ad.tile(m, n) - snap[Ad.offset(m, n):Ad.offset(m, n) + 1].new_tensor(0)).abs().max().item()
                tiles = [(m, n) for (m, n) in Ad.local_tiles()
                         if not torch.equal(Ad.tile(m, n), torch.as_strided(snap, Ad.tile(m, n).shape,
                                                                            Ad.tile(m, n).stride(), Ad.offset(m, n)))]
                print("   changed tiles", tiles[:20], flush=True)
        with B.predicated(1 - flag):
            tpd._qr_step(st, zero_ipiv=False)
        torch.cuda.synchronize()
        nan2 = bool(torch.isnan(Ad.data).any())
        # host path, same step
        sth = lu_qr._Step(Ah, k, p)
        mine = tph._domain_lu(sth)
        cond, piv = tph._decide(sth, mine)
        if cond:
            tph._lu_step(sth, mine, piv)
        else:
            tph._qr_step(sth)
        torch.cuda.synchronize()
        d = (Ad.data - Ah.data).abs().max().item()
        print(f"k={k} flag={int(flag.item())} host={cond} nan after LU-branch {nan1} after QR-branch {nan2} "
              f"max|A_dev - A_host| {d:.3e}", flush=True)
        if nan2 or d > 1e-8:
            dd = (Ad.data - Ah.data).abs()
            for (m, n) in Ad.local_tiles():
                e = (Ad.tile(m, n) - Ah.tile(m, n)).abs().max().item()
                if e > 1e-8 or torch.isnan(Ad.tile(m, n)).any():
                    print(f"   tile ({m},{n}) diff {e:.3e} nan {bool(torch.isnan(Ad.tile(m, n)).any())}")
            break


if __name__ == "__main__":
    main()
