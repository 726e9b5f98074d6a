"""Discrete-event model of the DTR push scheduler (csrc/kernels/dtr.hip k_dtr_q) on one MI355X.

  python tools/dtr_sim.py N [--wg 256] [--buckets B] [--weights upd1,upd_k,trsm,potrf] [--head 1,2] [--trace f.npz]

The plan and the ready-ring classes are the ones models/potrf_dtr.py builds (queue_plan); task durations are the
means measured by tools/gpu/dtr_trace_run.py at one workgroup per CU (UPD nk=1 ~76 us, nk=4 ~256 us, TRSM strip
~177 us; the 16 POTRF(k) blocks each end ~23 us after the previous one).  Idle workgroups pop the lowest non-empty
class, own XCD first, as the kernel does.  Used to compare priority schemes on the CPU before spending GPU time;
--trace checks the model against a measured trace (span, per-step POTRF starts).
"""
import argparse
import heapq
import os
import sys
from collections import deque
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

DUR = {"upd1": 76.0, "upd4_per_k": 64.0, "trsm": 177.0, "potrf_blk": 23.0, "pop": 4.0}


def simulate(plan, q, nwg=256, dur=DUR, prio=None, override=None):
    from dplasma_amd.models import potrf_dtr as D
    T = plan.tasks
    n = len(T)
    typ, nk, k0, blk = T["type"], T["nk"].astype(float), T["k0"], T["r"]
    d = np.where(typ == D.T_UPD, np.where(nk <= 1, dur["upd1"], dur["upd4_per_k"] * nk),
                 np.where(typ == D.T_TRSM, dur["trsm"], 0.0))
    if override is not None:   # (mask, duration): what-if durations of selected tasks
        d = np.where(override[0], override[1], d)
    pend = q["ndeps"].astype(np.int64).copy()
    so, su = q["succ_off"], q["succ"]
    ring = q["ring_of"] if prio is None else prio
    nring = int(ring.max()) + 1
    rings = [deque() for _ in range(nring)]
    nonempty = []                       # heap of ring ids with tasks (lazy)
    for t in np.nonzero(pend == 0)[0]:
        rings[ring[t]].append(t)
        heapq.heappush(nonempty, ring[t])
    ev = []                             # (time, seq, kind, worker, task)
    seq = 0
    idle = list(range(nwg))
    potrf_end = {}                      # (k, b) -> end time
    potrf_wait = {}                     # (k, b) -> (worker, start) started but waiting for block b-1
    start = np.full(n, -1.0)
    end = np.full(n, -1.0)
    now = 0.0

    def pop():
        while nonempty:
            r = nonempty[0]
            if rings[r]:
                t = rings[r].popleft()
                if not rings[r]:
                    heapq.heappop(nonempty)
                return t
            heapq.heappop(nonempty)
        return -1

    def begin(w, t, tnow):
        nonlocal seq
        ts = tnow + dur["pop"]
        start[t] = ts
        if typ[t] == D.T_POTRF:
            k, b = int(k0[t]), int(blk[t])
            if b == 0:
                e = ts + dur["potrf_blk"]
            elif (k, b - 1) in potrf_end:
                e = max(ts + dur["potrf_blk"], potrf_end[(k, b - 1)] + dur["potrf_blk"])
            else:
                potrf_wait[(k, b)] = (w, t, ts)
                return
            potrf_end[(k, b)] = e
            seq += 1
            heapq.heappush(ev, (e, seq, w, t))
            nxt = potrf_wait.pop((k, b + 1), None)
            if nxt is not None:
                begin_potrf_cont(nxt, k, b + 1, e)
            return
        seq += 1
        heapq.heappush(ev, (ts + d[t], seq, w, t))

    def begin_potrf_cont(rec, k, b, prev_end):
        nonlocal seq
        w, t, ts = rec
        e = max(ts + dur["potrf_blk"], prev_end + dur["potrf_blk"])
        potrf_end[(k, b)] = e
        seq += 1
        heapq.heappush(ev, (e, seq, w, t))
        nxt = potrf_wait.pop((k, b + 1), None)
        if nxt is not None:
            begin_potrf_cont(nxt, k, b + 1, e)

    def dispatch(tnow):
        while idle:
            t = pop()
            if t < 0:
                return
            begin(idle.pop(), t, tnow)

    dispatch(0.0)
    done = 0
    while ev:
        now, _, w, t = heapq.heappop(ev)
        end[t] = now
        done += 1
        for x in su[so[t]:so[t + 1]]:
            pend[x] -= 1
            if pend[x] == 0:
                rings[ring[x]].append(x)
                heapq.heappush(nonempty, ring[x])
        idle.append(w)
        dispatch(now + 2.0)
    if done != n:
        raise RuntimeError(f"simulation stalled: {done} of {n} tasks")
    return start, end


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("N", type=int, nargs="?", default=16384)
    ap.add_argument("--wg", type=int, default=256)
    ap.add_argument("--trace", default=None)
    ap.add_argument("--scheme", default="bl", help="bl (the kernel's classes) or exact (one class per distinct "
                                                     "bottom level: the unbucketed list-scheduling order)")
    a = ap.parse_args()
    from dplasma_amd.models import potrf_dtr as D
    nt = a.N // 512
    plan = D._Plan(nt, max(1, int(os.environ.get("DPLASMA_DTR_DEFER", "4"))), "column",
                   int(os.environ.get("DPLASMA_DTR_DEFER_MIN_TILES", "0")))
    q = D.queue_plan(plan)
    prio = None
    if a.scheme == "exact":
        bl = D.bottom_levels(q["succ_off"], q["succ"], D.task_weights(plan.tasks))
        T = plan.tasks
        order = np.argsort(-bl, kind="stable")
        prio = np.empty(len(T), dtype=np.int64)
        prio[order] = np.arange(len(T))
        prio = np.where(T["type"] == D.T_POTRF, 0, prio + 1)
    s, e = simulate(plan, q, a.wg, prio=prio)
    span = e.max()
    fl = a.N ** 3 / 3.0
    print(f"N={a.N} model span {span / 1e3:.2f} ms  ({fl / (span * 1e-6) / 1e12:.1f} TF/s)  buckets={D.UPD_BUCKETS} "
          f"scheme={a.scheme}")
    T = plan.tasks
    ps = [s[(T['type'] == D.T_POTRF) & (T['k0'] == k)].min() for k in range(nt)]
    print("POTRF starts (ms):", " ".join(f"{x / 1e3:.1f}" for x in ps[::max(1, nt // 16)]))
    if a.trace:
        d = np.load(a.trace)
        tr = d["trace"]
        t0 = tr[:, 0].min()
        ms = (tr[:, 1].max() - t0) / 100.0
        ty, kk = d["type"], d["k0"]
        mps = [(tr[(ty == 2) & (kk == k), 0].min() - t0) / 100.0 for k in range(nt)]
        print(f"measured span {ms / 1e3:.2f} ms")
        print("measured POTRF starts:", " ".join(f"{x / 1e3:.1f}" for x in mps[::max(1, nt // 16)]))


if __name__ == "__main__":
    main()
