#!/usr/bin/env python3
"""Critical-chain breakdown of a replayed rank's kernel trace (rocprofv3 --kernel-trace CSV of
tools/replay_potrf.py, one rank, warm-up + one timed run): per panel step of the timed run, the span from
one diagonal-tile POTRF (or the received-triangle prep) to the next, and how much of it the tile kernel,
the panel TRSM of this rank, the GEMM on the panel stream (NEAR / NEXT) and the bulk GEMM occupy.

python tools/replay_chain.py TRACE.csv"""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = []
    for r in rows:
        n = r["Kernel_Name"]
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        q = (r["Queue_Id"], r["Stream_Id"])
        kind = ("potrf" if "k_potrf_rb" in n else "prep" if "trsm_rb_prep" in n else "trsm" if "k_trsm_rb" in n
                else "gemm" if "k_gemm" in n else "delay" if "k_delay" in n else "other")
        ev.append((s, e, kind, q))
    ev.sort()
    # the timed run: the second half of the chain starts (potrf or prep) -- split at the largest gap
    starts = [x for x in ev if x[2] in ("potrf", "prep")]
    gaps = [(starts[i + 1][0] - starts[i][1], i) for i in range(len(starts) - 1)]
    cut = max(gaps)[1] + 1 if gaps else 0
    chain = starts[cut:]
    t0 = chain[0][0]
    t_end = max(e for s, e, k, q in ev if s >= t0)
    # stream of the panel GEMMs: the gemm queue that carries the fewest flops... use stream ids
    qs = defaultdict(float)
    for s, e, k, q in ev:
        if k == "gemm" and s >= t0:
            qs[q] += e - s
    print(f"timed run: {(t_end - t0) / 1e6:.2f} ms, {len(chain)} chain heads; gemm busy per queue (ms):",
          {str(k): round(v / 1e6, 1) for k, v in qs.items()})
    tot = defaultdict(float)
    print(" step  span(us)  tile  trsm(own)  gemm-overlap  delay")
    for i in range(len(chain) - 1):
        a, b = chain[i][0], chain[i + 1][0]
        acc = defaultdict(float)
        for s, e, k, q in ev:
            if e <= a or s >= b:
                continue
            acc[k] += min(e, b) - max(s, a)
        span = b - a
        for k, v in acc.items():
            tot[k] += v
        tot["span"] += span
        if i % 8 == 0:
            print(f" {i:4d} {span / 1e3:9.1f} {acc['potrf'] / 1e3 + acc['prep'] / 1e3:6.1f} {acc['trsm'] / 1e3:9.1f}"
                  f" {acc['gemm'] / 1e3:12.1f} {acc['delay'] / 1e3:7.1f}")
    print("totals (ms):", {k: round(v / 1e6, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()
