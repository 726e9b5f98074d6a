"""Why a push-scheduled grid emulation stalls: counters / rings after the drain."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import dplasma_amd as dp  # noqa: E402
from dplasma_amd.models import potrf_dtr as D  # noqa: E402
from dplasma_amd.models import potrf_dtr_dist as DD  # noqa: E402


def main():
    N, P, Q = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    ctx = dp.init()
    em = DD.Emulation(ctx, N, P, Q, bw_gbs=50.0, lat_us=10.0)
    em.reset()
    print("img rank", em.img.buf[em.img.off["rank"]:em.img.off["rank"] + 4], "nranks",
          em.img.buf[em.img.off["nranks"]:em.img.off["nranks"] + 4], "rdy ptr", em.qk["rdy"].data_ptr(),
          int.from_bytes(em.img.buf[em.img.off["rdy"]:em.img.off["rdy"] + 8], "little"), flush=True)
    try:
        em.run()
        print("run ok", flush=True)
    except RuntimeError as e:
        print("error", e, flush=True)
    qk = em.qk
    plan = em.plan
    done = int(qk["done"].item())
    print("done", done, "of", len(plan.tasks), flush=True)
    nring = D.NCLASS * 8
    typ = plan.tasks["type"]
    for r in range(em.nr):
        pend = qk["pend"][r].cpu().numpy()
        mine = plan.owner == r
        left = np.nonzero(mine & (pend > 0))[0]
        print(f"rank {r}: tasks {mine.sum()} pending>0 {len(left)} types {np.bincount(typ[left], minlength=5)}", flush=True)
        ctl = qk["qctl"][r].cpu().numpy().reshape(nring, 2, -1)[:, :, 0]
        nz = [(q, int(ctl[q, 0]), int(ctl[q, 1])) for q in range(nring) if ctl[q, 1] != ctl[q, 0]]
        print("   rings with work (ring, head, tail):", nz[:12], flush=True)
        qs = qk["qslot"][r].cpu().numpy()
        qb = qk["qbase"].cpu().numpy()[r * (nring + 1):(r + 1) * (nring + 1)]
        rdy = qk["rdy"].cpu().numpy()
        for (q, h, tl) in nz[:4]:
            sl = qs[qb[q]:qb[q] + tl]
            print(f"   ring {q}: base {qb[q]} slots {sl.tolist()} pend {[int(pend[x - 1]) for x in sl if x]} "
                  f"rdy {[int(rdy[x - 1]) for x in sl if x]} types {[int(typ[x - 1]) for x in sl if x]}", flush=True)
        # tasks that are ready (pend 0) but never completed? (pushed and not popped)
    rdy = qk["rdy"].cpu().numpy()
    print("rdy max", rdy.max(), flush=True)


if __name__ == "__main__":
    main()
