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
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    ks.sort()
    t0 = [s for s, e, n in ks if args.from_kernel in n][args.skip]
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


if __name__ == "__main__":
    main()
