"""Repeat one DTR Cholesky configuration and residual-check every run (intermittent-failure hunt).

  python tools/gpu/dtr_repeat.py N runs

DPLASMA_DTR_PROBE=1: also print the strip-hazard probe's records of every run (csrc/kernels/dtr.hip probe_strip:
kind 1 = a diagonal-tile update started before its strip's TRSM stamp, kind 2 = a strip read differently through
the CU's caches than from memory).
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import dplasma_amd as dp  # noqa: E402
from dplasma_amd.models import potrf_dtr as D  # noqa: E402


def main():
    N, runs = int(sys.argv[1]), int(sys.argv[2])
    ctx = dp.init()
    A = dp.block_cyclic(ctx, torch.float64, 512, 512, N, N)
    dp.dplghe(ctx, float(N), dp.dplasmaLower, A, 3872)
    A0 = A.data.clone()
    tp = D.potrf_dtr_New(ctx, dp.dplasmaLower, A)
    Ar = A.like()
    bad = 0
    good = None
    nt = N // 512
    probe = getattr(tp, "dtr_probe", None)
    nprobe = [0] * 7
    for rep in range(runs):
        A.data.copy_(A0)
        tp.info.zero_()
        if probe is not None:
            probe[0] = 0
        tp.execute(ctx)
        info = int(tp.info.item())
        # every counter at its final value (a task run twice would leave one above it)
        plan = tp.dtr_plan
        cnt = tp._keep[5].cpu().numpy()
        exp = np.concatenate([plan.final_ver, np.full(plan.nt, 16)]).astype(np.int64)
        over = np.nonzero(cnt.astype(np.int64) != exp)[0]
        cmsg = f" counters off: {len(over)} e.g. {[(int(q), int(cnt[q]), int(exp[q])) for q in over[:6]]}" if len(over) else ""
        L = torch.tril(A.to_dense_local())
        Ar.data.copy_(A0)
        ok, res = dp.check_potrf(ctx, dp.dplasmaLower, A, Ar)
        bad += not ok
        msg = ""
        if ok and good is None:
            good = L.clone()
        elif not ok and good is not None:
            # 128 x 128 sub-tiles that differ from a good run's factor, in factorisation order (k, i, r, c)
            d = (L - good).abs().view(nt, 4, 128, nt, 4, 128).amax(dim=(2, 5))   # [i, r, j, c]
            idx = torch.nonzero(d > 1e-9)
            lst = sorted((int(j), int(i), int(r), int(c), float(d[i, r, j, c])) for i, r, j, c in idx.tolist())
            msg = f" info={info} bad sub-tiles {len(lst)} first (j, i, r, c, err): {lst[:8]}"
            snap = getattr(tp, "dtr_snap", None)
            if snap is not None and lst:
                # the first wrong diagonal tile: was POTRF's input wrong, or its factorisation of that input?
                j0 = lst[0][0]
                inp = torch.tril(snap[j0 * 512 * 512:(j0 + 1) * 512 * 512].view(512, 512).t()).cpu()
                lj = L[j0 * 512:(j0 + 1) * 512, j0 * 512:(j0 + 1) * 512].cpu()
                lh = torch.linalg.cholesky(inp + torch.tril(inp, -1).t())
                gin = good[j0 * 512:(j0 + 1) * 512, j0 * 512:(j0 + 1) * 512].cpu()
                msg += (f" | tile {j0}: |out - chol(input)| = {float((lj - lh).abs().max()):.2e}, "
                        f"|out - good| = {float((lj - gin).abs().max()):.2e}, |chol(input) - good| = "
                        f"{float((lh - gin).abs().max()):.2e}")
                # which 32 x 32 blocks (row block i, column block k) of the tile's factor are wrong, in dataflow order
                e32 = (torch.tril(lj) - lh).abs().view(16, 32, 16, 32).amax(dim=(1, 3))
                bad32 = sorted((int(k_), int(i_), float(e32[i_, k_])) for i_, k_ in torch.nonzero(e32 > 1e-9).tolist())
                msg += f"; wrong 32-blocks (k, i, err) {[(a_, b_, f'{c_:.1e}') for a_, b_, c_ in bad32[:10]]}"
                # post mortem of the tile's published hand-off blocks (PotrfScratch, per tile, intact after the run):
                # Lp(i, k) (L(i,k) as published for the row blocks below) vs the factor's own L(i,k) in A, and
                # Z_k = diag(S_k) M_k vs inv(L(k,k))
                scr = tp._keep[10]
                MAXB, BLK = 16, 1024
                w_, r_, l_ = np.meshgrid(np.arange(16) // 4, np.arange(16) % 4, np.arange(64), indexing="ij")
                e_idx = (np.arange(16)[:, None] * 64 + np.arange(64)[None, :]).ravel()
                ww, rr, ll = (np.arange(16) // 4)[:, None].repeat(64, 1).ravel(), (np.arange(16) % 4)[:, None].repeat(64, 1).ravel(), np.tile(np.arange(64), 16)
                rho = 16 * (ww >> 1) + (ll & 15)
                gam = 16 * (ww & 1) + (ll >> 4) + 4 * rr
                Lp = scr.Lp[j0 * MAXB * MAXB * BLK:(j0 + 1) * MAXB * MAXB * BLK].view(MAXB, MAXB, BLK).cpu()
                lpbad = []
                for i_ in range(1, 16):
                    for k_ in range(i_):
                        blk = torch.zeros(32, 32, dtype=torch.float64)
                        blk[rho, gam] = Lp[i_, k_][e_idx]
                        ref = lj[32 * i_:32 * i_ + 32, 32 * k_:32 * k_ + 32]
                        d_ = float((blk - ref).abs().max())
                        if d_ > 1e-9:
                            lpbad.append((i_, k_, f"{d_:.1e}"))
                Mw = scr.Mw[j0 * MAXB * BLK:(j0 + 1) * MAXB * BLK].view(MAXB, 32, 32).cpu()   # [k][col][row]
                Sw = scr.Sw[j0 * MAXB * 32:(j0 + 1) * MAXB * 32].view(MAXB, 32).cpu()
                zbad = []
                for k_ in range(16):
                    Z = torch.diag(Sw[k_]) @ Mw[k_].t()
                    Lkk = lj[32 * k_:32 * k_ + 32, 32 * k_:32 * k_ + 32]
                    d_ = float((Z @ Lkk - torch.eye(32, dtype=torch.float64)).abs().max())
                    if d_ > 1e-8:
                        zbad.append((k_, f"{d_:.1e}"))
                msg += f"; published L blocks wrong (i, k, err) {lpbad[:8]} of {len(lpbad)}; Z_k wrong {zbad[:6]}"
        pmsg = ""
        if probe is not None:
            pr = probe.cpu().numpy()
            n = int(min(pr[0], 4096))
            recs = pr[8 + 20 * nt * nt: 8 + 20 * nt * nt + 8 * n].reshape(n, 8)
            kinds = [int(x & 15) for x in recs[:, 1]]
            for kd in range(1, 7):
                nprobe[kd] += kinds.count(kd)
            if n:
                show = [(int(r_[0]), int(r_[1] >> 16), int((r_[1] >> 8) & 255), int((r_[1] >> 4) & 15), int(r_[1] & 15),
                         int(r_[2] >> 8), int(r_[2] & 255), int(r_[3]),
                         float(np.frombuffer(np.int64(r_[4]).tobytes())[0]), float(np.frombuffer(np.int64(r_[5]).tobytes())[0]))
                        for r_ in recs[:6]]
                pmsg = (f" probe: {n} records by kind {[kinds.count(kd) for kd in range(1, 7)]}; first (task, "
                        f"k|tile, strip|sub, phase, kind, wg, xcd, stamp, plain, mem): {show}")
        print(f"run {rep}: check={ok} res={res:.2e}{msg}{cmsg}{pmsg}", flush=True)
    print(f"FAILED {bad} / {runs}" + (f"; probe records by kind (1 strip stamp, 2 strip cache, 3 C stamp, 4 C cache, "
                                      f"5 POTRF-input stamp, 6 POTRF-input cache): {nprobe[1:]}"
                                      if probe is not None else ""), flush=True)


if __name__ == "__main__":
    main()
