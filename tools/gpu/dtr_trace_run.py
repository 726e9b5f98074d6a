"""Per-task timeline of the device task runtime Cholesky (DPLASMA_DTR_TRACE=1).

  python tools/gpu/dtr_trace_run.py N [out.npz]

Prints, per task kind, the count and the mean / total duration; the workgroup occupancy (busy time
over 2 x #CUs workgroups x span); and per panel k the critical chain: POTRF(k) span (first start of
its 16 workgroups -> last end), its TRSM strips' span, and the gap from the last update of column k+1
to POTRF(k+1)'s start.
"""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
os.environ["DPLASMA_DTR_TRACE"] = "1"
import numpy as np  # noqa: E402
import torch  # noqa: E402

import dplasma_amd as dp  # noqa: E402
from dplasma_amd.models import potrf_dtr as D  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    out = sys.argv[2] if len(sys.argv) > 2 else None
    ctx = dp.init()
    A = dp.block_cyclic(ctx, torch.float64, 512, 512, N, N)
    dp.dplghe(ctx, float(N), dp.dplasmaLower, A, 3872)
    A0 = A.data.clone()
    tp = D.potrf_dtr_New(ctx, dp.dplasmaLower, A)
    # DTR_TRACE_RUNS=n: up to n runs, stopping at the first whose residual check fails (that run's trace is kept)
    runs = int(os.environ.get("DTR_TRACE_RUNS", "2"))
    for rep in range(runs):
        A.data.copy_(A0)
        tp.dtr_trace.zero_()
        tp.execute(ctx)
        if runs > 2:
            Ar = A.like()
            Ar.data.copy_(A0)
            ok, res = dp.check_potrf(ctx, dp.dplasmaLower, A, Ar)
            print(f"run {rep}: check={ok} res={res:.2e}", flush=True)
            if not ok:
                break
    torch.cuda.synchronize()
    tr = tp.dtr_trace[:4 * len(tp.dtr_plan.tasks)].view(-1, 4).cpu().numpy()
    ph = tp.dtr_trace[4 * len(tp.dtr_plan.tasks):].view(-1, 16, 64).cpu().numpy()
    plan = tp.dtr_plan
    T = plan.tasks
    s, e, who = tr[:, 0], tr[:, 1], tr[:, 2]
    t0 = s.min()
    span = (e.max() - t0) / 100.0   # us
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    nwg = 2 * ncu
    dur = (e - s) / 100.0
    print(f"N={N} tasks={len(T)} span={span / 1e3:.2f} ms  ({tp.flops / (span * 1e-6) / 1e12:.2f} TF/s)")
    names = {D.T_UPD: "UPD", D.T_TRSM: "TRSM", D.T_POTRF: "POTRF"}
    busy = dur.sum()
    print(f"workgroup occupancy: {busy / (nwg * span) * 100:.1f} % of {nwg} workgroups x span")
    for ty, nm in names.items():
        m = T["type"] == ty
        if ty == D.T_UPD:
            for nk in sorted(set(T["nk"][m].tolist())):
                mm = m & (T["nk"] == nk)
                print(f"  {nm}(nk={nk}): {mm.sum():8d} tasks  mean {dur[mm].mean():8.1f} us  total {dur[mm].sum() / 1e3:9.1f} ms")
        else:
            print(f"  {nm:9s}: {m.sum():8d} tasks  mean {dur[m].mean():8.1f} us  total {dur[m].sum() / 1e3:9.1f} ms")
    # per-panel chain
    nt = plan.nt
    print(" k | POTRF start..end (us from t0) | TRSM first..last end | wait before POTRF")
    prev_end = 0.0
    for k in range(min(nt, 24)):
        mp = (T["type"] == D.T_POTRF) & (T["k0"] == k)
        mt_ = (T["type"] == D.T_TRSM) & (T["k0"] == k)
        ps, pe = (s[mp].min() - t0) / 100.0, (e[mp].max() - t0) / 100.0
        ts_, te = ((s[mt_].min() - t0) / 100.0, (e[mt_].max() - t0) / 100.0) if mt_.any() else (pe, pe)
        print(f"{k:3d} | {ps:10.1f} .. {pe:10.1f} ({pe - ps:7.1f}) | {ts_:10.1f} .. {te:10.1f} ({te - ts_:7.1f}) | "
              f"{ps - prev_end:8.1f}")
        prev_end = te
    # occupancy over time (20 bins) and the share of idle workgroup-time in the first / last fifth
    nb_ = 20
    edges = np.linspace(0, span, nb_ + 1)
    ss, ee = (s - t0) / 100.0, (e - t0) / 100.0
    occ = []
    for q in range(nb_):
        lo, hi = edges[q], edges[q + 1]
        busy_q = np.clip(np.minimum(ee, hi) - np.maximum(ss, lo), 0, None).sum()
        occ.append(int(round(100 * busy_q / (nwg * (hi - lo)))))
    print("occupancy per 5 % of the span:", occ)
    # gaps between consecutive tasks of each workgroup: many small ones = per-task overhead, few large ones =
    # stalls; split by the kind of the task that follows the gap and by XCD
    wg_of, xcd_of = who >> 8, who & 0xff
    order = np.lexsort((ss, wg_of))
    wo, so, eo = wg_of[order], ss[order], ee[order]
    same = wo[1:] == wo[:-1]
    gaps = (so[1:] - eo[:-1])[same]
    nxt = order[1:][same]
    tot = gaps.sum()
    print(f"gaps: n={len(gaps)} total {tot / 1e3:.1f} WG-ms ({100 * tot / (nwg * span):.1f} % of WG x span)  mean {gaps.mean():.1f} us"
          f"  p50 {np.percentile(gaps, 50):.1f}  p90 {np.percentile(gaps, 90):.1f}  p99 {np.percentile(gaps, 99):.1f}")
    for lo_, hi_ in ((0, 5), (5, 20), (20, 100), (100, 1000), (1000, 1e12)):
        m = (gaps >= lo_) & (gaps < hi_)
        print(f"  gaps in [{lo_}, {hi_}) us: {m.sum():8d}  sum {gaps[m].sum() / 1e3:9.1f} WG-ms")
    hi_set = np.zeros(len(T), dtype=bool)
    hi_set[plan.hi] = True
    for nm, m in (("next task from the high list", hi_set[nxt]), ("next task from a low list", ~hi_set[nxt])):
        print(f"  {nm}: {m.sum()} gaps, {gaps[m].sum() / 1e3:.1f} WG-ms")
    xb = [(ee[xcd_of == x] - ss[xcd_of == x]).sum() / ((nwg / 8) * span) * 100 for x in range(8)]
    print("busy % per XCD:", [int(round(v)) for v in xb])
    if out:
        np.savez(out, trace=tr, tasks=T.view(np.uint8), nt=nt, owner=np.zeros(len(T), dtype=np.int64),
                 type=T["type"], k0=T["k0"], i=T["i"], j=T["j"], r=T["r"], nk=T["nk"], inc=T["inc"], req_beg=T["req_beg"],
                 nreq=T["nreq"], reqs=plan.reqs, nranks=1, phase=ph)

    # POTRF(k) phases per block (us from the step's first block start): factor chain end (slot 51), W column end (53)
    for k in list(range(min(6, nt))) + [nt // 2, nt - 1]:
        p = ph[k].astype(np.float64)
        b0 = p[:, 0].min()
        st = (p[:, 0] - b0) / 100.0
        dg = (p[:, 49] - b0) / 100.0
        fe = (p[:, 51] - b0) / 100.0
        we = (p[:, 53] - b0) / 100.0
        print(f"POTRF({k}) block start " + " ".join(f"{x:.0f}" for x in st))
        print(f"   diag start  " + " ".join(f"{x:.0f}" for x in dg))
        print(f"   factor end  " + " ".join(f"{x:.0f}" for x in fe))
        print(f"   W end       " + " ".join(f"{x:.0f}" for x in we))


if __name__ == "__main__":
    main()
