#!/usr/bin/env python3
"""Critical chain of an emulated P x Q DTR Cholesky trace (tools/emulate_potrf.py --trace out.npz).

Per panel k (times in modelled microseconds = emulated ticks / (P Q) / 100): POTRF(k) on its owner
(first start .. last end), the TRSM strips of tile (k+1, k) (on owner(k+1, k)), the SENDs of those strips
to owner(k+1, k+1), the diagonal updates of tile (k+1, k+1) by panel k, and POTRF(k+1)'s start.  Also per
rank: busy fraction of its workgroups, and per task kind counts / mean durations.

  python tools/emul_trace.py out.npz P Q [kmax]
"""
import sys

import numpy as np

T_UPD, T_TRSM, T_POTRF, T_SEND, T_SENDW = 0, 1, 2, 3, 4
NAMES = {0: "UPD", 1: "TRSM", 2: "POTRF", 3: "SEND", 4: "SENDW"}


def main():
    z = np.load(sys.argv[1])
    P, Q = int(sys.argv[2]), int(sys.argv[3])
    kmax = int(sys.argv[4]) if len(sys.argv) > 4 else 24
    nr = P * Q
    tr, own, ty, k0, ti, tj = z["trace"], z["owner"], z["type"], z["k0"], z["i"], z["j"]
    s, e = tr[:, 0].astype(np.int64), tr[:, 1].astype(np.int64)
    ran = e > 0
    t0 = s[ran].min()
    scale = 100.0 * nr            # ticks -> modelled us
    S = (s - t0) / scale
    E = (e - t0) / scale
    span = E[ran].max()
    print(f"span {span / 1e3:.2f} ms modelled, tasks {ran.sum()} / {len(ran)}")
    wg = tr[:, 2] >> 8
    for r in range(nr):
        m = ran & (own == r)
        nwg = len(np.unique(wg[m]))
        busy = (E[m] - S[m]).sum() / (span * max(nwg, 1))
        kinds = ", ".join(f"{NAMES[k]} {int((m & (ty == k)).sum())} x {np.mean(E[m & (ty == k)] - S[m & (ty == k)]):.0f}us"
                          for k in range(5) if (m & (ty == k)).any())
        print(f" rank {r}: {nwg} wgs, busy {100 * busy:.1f} %  [{kinds}]")

    def owner(i, j):
        return (i % P) * Q + (j % Q)
    print(" k | POTRF(k)            | TRSM(k+1,k)          | SEND->diag | UPD diag   | next POTRF")
    for k in range(min(kmax, int(k0.max()))):
        po = (ty == T_POTRF) & (k0 == k) & ran
        tr_ = (ty == T_TRSM) & (k0 == k) & (ti == k + 1) & ran
        d = owner(k + 1, k + 1)
        sd = (ty == T_SEND) & (k0 == k) & (ti == k + 1) & (tj == d) & ran
        ud = (ty == T_UPD) & (ti == k + 1) & (tj == k + 1) & (k0 <= k) & (k0 + z.get("nk", np.ones_like(k0)) > k) & ran \
            if "nk" in z else (ty == T_UPD) & (ti == k + 1) & (tj == k + 1) & ran
        pn = (ty == T_POTRF) & (k0 == k + 1) & ran
        f = lambda m: f"{S[m].min():8.0f}..{E[m].max():8.0f}" if m.any() else "        -         "  # noqa: E731
        print(f"{k:3d} | {f(po)} | {f(tr_)} | {E[sd].max() if sd.any() else float('nan'):9.0f} | "
              f"{f(ud)} | {S[pn].min() if pn.any() else float('nan'):9.0f}")


if __name__ == "__main__":
    main()
