#!/usr/bin/env python3
"""Critical path of a DTR run from its task trace (tools/emulate_potrf.py --trace, or the 1-GPU trace).

For every task, the producer of each requirement is the bump that made the counter reach its target on
the task's rank (bumps ordered by the time they became visible: the emulation's dilated visibility, the
end time otherwise); the critical predecessor is the requirement that became visible last.  Walking back
from the last task gives the chain that set the span; each hop is split into the time the task waited
after its last input became visible (list order, no free workgroup, ticket races) and the time it took
(effective: until its own completion became visible).

  python tools/emul_critical.py trace.npz [ranks] [show]
"""
import sys
from collections import defaultdict

import numpy as np

NAMES = {0: "UPD", 1: "TRSM", 2: "POTRF", 3: "SEND", 4: "SENDW"}


def main():
    z = np.load(sys.argv[1])
    nr = int(sys.argv[2]) if len(sys.argv) > 2 else int(z["nranks"]) if "nranks" in z else 1
    show = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    tr = z["trace"]
    s, e = tr[:, 0].astype(np.int64), tr[:, 1].astype(np.int64)
    vis = tr[:, 3].astype(np.int64) if tr.shape[1] > 3 else e.copy()
    if nr == 1:    # one process: column 3 counts the executions of each task
        runs = vis.copy()
        print(f"executions per task: min {runs.min()} max {runs.max()} (tasks run != 1: {(runs != 1).sum()})")
        vis = e.copy()
    vis = np.where(vis > 0, vis, e)
    ty, own, inc, tj = z["type"], z["owner"], z["inc"], z["j"]
    rb, nrq, reqs = z["req_beg"], z["nreq"], z["reqs"]
    t0 = s[e > 0].min()
    sc = 100.0 * nr                     # ticks -> modelled us
    tgt = np.where((ty == 3) | (ty == 4), tj, own)
    bumps = defaultdict(list)
    for t in np.nonzero(inc >= 0)[0]:
        bumps[(int(tgt[t]), int(inc[t]))].append((int(vis[t]), int(t)))
    for k in bumps:
        bumps[k].sort()

    def crit_pred(t):
        r = int(own[t])
        best, bt = -1, -1
        for q in range(int(rb[t]), int(rb[t]) + int(nrq[t])):
            c, target = int(reqs[q, 0]), int(reqs[q, 1])
            lst = bumps.get((r, c), [])
            if target <= 0 or target > len(lst):
                continue
            v, p = lst[target - 1]
            if v > best:
                best, bt = v, p
        return bt, best
    # dependency check: a task must start after every input it required became visible
    viol = 0
    for t in range(len(s)):
        p, pv = crit_pred(t)
        if p >= 0 and pv > s[t] + 200:       # 2 us of clock skew between XCDs tolerated
            if viol < 10:
                print(f"VIOLATION: {NAMES[int(ty[t])]} i={int(z['i'][t])} j={int(z['j'][t])} k0={int(z['k0'][t])} "
                      f"r={int(z['r'][t]) if 'r' in z else -1} started {(pv - s[t]) / 100:.1f} us before its input "
                      f"{NAMES[int(ty[p])]} i={int(z['i'][p])} j={int(z['j'][p])} k0={int(z['k0'][p])} was visible")
            viol += 1
    print(f"dependency violations: {viol}")
    t = int(np.argmax(vis))
    path = []
    while t >= 0:
        p, pv = crit_pred(t)
        path.append((t, p, pv))
        t = p
    path.reverse()
    wait = defaultdict(float)
    eff = defaultdict(float)
    for t, p, pv in path:
        w = (s[t] - pv) / sc if p >= 0 else (s[t] - t0) / sc
        wait[NAMES[int(ty[t])]] += max(w, 0)
        eff[NAMES[int(ty[t])]] += (vis[t] - s[t]) / sc
    span = (vis.max() - t0) / sc
    print(f"span {span / 1e3:.2f} ms modelled; critical path: {len(path)} tasks")
    for k in sorted(eff):
        print(f"  {k:6s} effective {eff[k] / 1e3:8.2f} ms   waited before start {wait[k] / 1e3:8.2f} ms")
    print(" hop | task                          | rank | wait us | effective us")
    step = max(1, len(path) // show)
    for n, (t, p, pv) in enumerate(path):
        if n % step and n != len(path) - 1:
            continue
        w = (s[t] - pv) / sc if p >= 0 else 0.0
        print(f"{n:4d} | {NAMES[int(ty[t])]:5s} i={int(z['i'][t]):3d} j={int(z['j'][t]):3d} k0={int(z['k0'][t]):3d} "
              f"nk={int(z['nk'][t]) if 'nk' in z else 0} | {int(own[t]):4d} | {w:7.0f} | {(vis[t] - s[t]) / sc:7.0f}")


if __name__ == "__main__":
    main()
