"""Summaries of a rocprofv3 SQLite result (``--kernel-trace`` without ``-f csv``).

python tools/prof_db.py gpurun_out/prof_qr/run_results.db [--top 15] [--timeline NAME_SUBSTR]
Prints per-kernel totals, the union of busy time, and optionally per-launch durations of one
kernel together with the gap to the previous launch on its queue (critical-path evidence)."""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--timeline", default=None)
    ap.add_argument("--skip", type=int, default=0, help="ignore launches before the N-th launch of --window")
    ap.add_argument("--window", default=None, help="restrict to [first, last] launch of this kernel substring")
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    rows = cur.execute("select name, start, end, queue_id from kernels order by start").fetchall()
    if a.window:
        idx = [i for i, r in enumerate(rows) if a.window in r[0]]
        if idx:
            rows = rows[idx[min(a.skip, len(idx) - 1)]: idx[-1] + 1]
    tot, cnt = defaultdict(int), defaultdict(int)
    for n, s, e, q in rows:
        short = n.split("(")[0][:90]
        tot[short] += e - s
        cnt[short] += 1
    t0, t1 = rows[0][1], max(r[2] for r in rows)
    busy, cs, ce = 0, None, None
    for _, s, e, _ in rows:
        if cs is None or s > ce:
            if cs is not None:
                busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    allk = sum(tot.values())
    print(f"window {(t1 - t0) / 1e6:.2f} ms, GPU busy (union) {busy / 1e6:.2f} ms, kernel sum {allk / 1e6:.2f} ms")
    for n, t in sorted(tot.items(), key=lambda x: -x[1])[: a.top]:
        print(f"{t / 1e6:10.2f} ms {100 * t / allk:5.1f}% {cnt[n]:7d} x {t / cnt[n] / 1e3:9.1f} us  {n}")
    if a.timeline:
        last = {}
        print("launch  dur(us)  gap_prev_same_queue(us)")
        for n, s, e, q in rows:
            if a.timeline in n:
                g = (s - last[q]) / 1e3 if q in last else 0.0
                print(f"{(s - t0) / 1e6:9.3f} ms {(e - s) / 1e3:9.1f} {g:9.1f}")
            last[q] = e


if __name__ == "__main__":
    main()
