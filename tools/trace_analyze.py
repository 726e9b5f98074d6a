#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (``*_kernel_trace.csv``) over a time window.

python tools/trace_analyze.py TRACE.csv [--from-kernel k_potrf] [--to-last k_potrf]

Prints, for the window [first dispatch whose name matches --from-kernel, end of the last
kernel], the busy time of each kernel class, the union of GEMM-engine intervals (how much
of the wall the flop engine is running) and the "exposed" time where no GEMM runs (the
critical-path cost that lookahead failed to hide).
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name):
    m = re.match(r"(?:void )?([A-Za-z_0-9:]+)(<[^>]*>)?", name)
    base = m.group(1) if m else name[:40]
    if base.startswith("at::native"):
        return "torch:" + base.split("::")[-1][:30]
    return base + (m.group(2) or "" if m else "")


def union(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--from-kernel", default="k_potrf")
    ap.add_argument("--engine", default="k_gemm")
    ap.add_argument("--skip", type=int, default=0, help="start at the (skip+1)-th --from-kernel dispatch")
    ap.add_argument("--last", action="store_true", help="start at the last run: the first --from-kernel "
                    "dispatch after the longest gap with no kernel (a host-side pause between runs)")
    ap.add_argument("--slices", type=int, default=0, help="also print engine busy / exposed time per time slice")
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    ks.sort()
    starts = [s for s, e, n in ks if args.from_kernel in n]
    t0 = starts[args.skip]
    if args.last:
        # the longest idle gap separates runs; take the first matching dispatch after it
        best, gap_end = -1, ks[0][0]
        run_end = ks[0][1]
        for s, e, n in ks[1:]:
            if s - run_end > best:
                best, gap_end = s - run_end, s
            run_end = max(run_end, e)
        t0 = min(x for x in starts if x >= gap_end)
    win = [(s, e, n) for s, e, n in ks if s >= t0]
    t1 = max(e for s, e, n in win)
    wall = t1 - t0
    busy = defaultdict(int)
    cnt = defaultdict(int)
    for s, e, n in win:
        busy[short(n)] += e - s
        cnt[short(n)] += 1
    eng = union([(s, e) for s, e, n in win if args.engine in n])
    anyk = union([(s, e) for s, e, n in win])
    print(f"window {wall / 1e6:.2f} ms; any-kernel union {anyk / 1e6:.2f} ms; engine union {eng / 1e6:.2f} ms; "
          f"exposed (no engine kernel running) {(wall - eng) / 1e6:.2f} ms")
    for k, v in sorted(busy.items(), key=lambda x: -x[1]):
        print(f"  {v / 1e6:10.2f} ms  {cnt[k]:6d}x  {k}")
    if args.slices:
        w = wall / args.slices
        print(f"per slice of {w / 1e6:.2f} ms: engine busy / exposed")
        for i in range(args.slices):
            a, b = t0 + i * w, t0 + (i + 1) * w
            e_ = union([(max(s, a), min(e, b)) for s, e, n in win if args.engine in n and e > a and s < b])
            print(f"  [{i * w / 1e6:7.2f}, {(i + 1) * w / 1e6:7.2f}) ms  engine {e_ / 1e6:6.2f}  exposed {(w - e_) / 1e6:6.2f}")


if __name__ == "__main__":
    main()
