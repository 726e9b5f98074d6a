#!/usr/bin/env python3
"""Timeline model of the distributed DPOTRF schedule (models/potrf.py) on P x Q MI355X GPUs.

A discrete-event simulation of the exact task structure potrf_New builds (blocks of D panels,
POTRF / DBCAST / TRSM / PANEL_COMM / NEAR on the high-priority panel stream, NEXT / REST on the
update stream, cross-rank edges through the panel broadcasts), fed with kernel costs measured on one
MI355X and an xGMI message model:

* GEMM (k_gemm_full): flops / R, R = 74.6 TF/s for launches that fill the chip, scaled down by
  workgroup count below two waves of workgroups (profiles/r1_kbench_gemm_full.txt);
* tile POTRF (k_potrf_rb): 185 us alone; TRSM (k_trsm_rb): 40 us + 100 us per round of 1024
  16-row strips, alone (profiles/r2_potrf16k_timeline.txt);
* contention: a panel kernel that starts while a bulk GEMM of the same GPU is running takes
  ``slow_potrf`` / ``slow_trsm`` times longer (16k trace: 3-7x and 10-28x);
* messages: latency + bytes / bandwidth per broadcast / all-gather (RCCL over xGMI; the
  bandwidth per transfer is a parameter -- one xGMI link is ~64 GB/s per direction).

It is a model, not a measurement: ``--calibrate`` prints its 1-GPU predictions next to the measured
16k / 32k / 64k times so the error of the cost model is visible.

  python tools/sim_potrf.py [-N 65536] [--nb 512] [--grids 1x1,1x2,2x2,2x4] [--bw 50] [--calibrate]
"""
from __future__ import annotations

import argparse
import heapq
from collections import defaultdict

MEASURED_1GPU = {16384: 0.03196, 32768: 0.18869, 65536: 1.34242}   # s, profiles/r2_bench_driver_cmd.txt & sweeps
PEAK = 78.6e12


class Model:
    def __init__(self, gemm_rate=74.6e12, t_potrf=185e-6, trsm_fixed=40e-6, trsm_round=100e-6,
                 slow_potrf=4.0, slow_trsm=12.0, lat=20e-6, bw=50e9, launch=8e-6):
        self.__dict__.update(locals())
        del self.__dict__["self"]

    def gemm(self, flops, wgs):
        if flops <= 0:
            return 0.0
        fill = min(1.0, wgs / 512.0)
        return self.launch + flops / (self.gemm_rate * max(fill, 0.05))

    def trsm(self, ntiles, nb):
        """k_trsm_rb: one wave per 16-row strip, ~1024 strips resident at once, ~100 us per round
        (16k trace: 31 tiles = 992 strips in 135-144 us)."""
        if not ntiles:
            return 0.0
        rounds = -(-(ntiles * nb // 16) // 1024)
        return self.trsm_fixed + rounds * self.trsm_round

    def msg(self, nbytes):
        return self.lat + nbytes / self.bw if nbytes > 0 else 0.0


def simulate(N, NB, P, Q, m: Model, D=4, min_tiles=24):
    nt = -(-N // NB)
    tile_b = NB * NB * 8
    ranks = [(p, q) for p in range(P) for q in range(Q)]
    blocks, c = [], 0
    while c < nt:
        d = D if nt - c >= min_tiles else 1
        blocks.append((c, min(nt, c + d)))
        c += d
    # stream availability per rank, task finish times, update-stream busy intervals
    free = {(r, s): 0.0 for r in ranks for s in ("panel", "update")}
    busy_upd = defaultdict(list)   # rank -> [(start, end)] of bulk GEMMs

    def overlapped(r, t0):
        return any(a <= t0 < b for a, b in busy_upd[r][-3:])

    def run(r, stream, ready, dur):
        t0 = max(free[(r, stream)], ready)
        t1 = t0 + dur
        free[(r, stream)] = t1
        return t0, t1

    own = lambda i, j: (i % P, j % Q)  # noqa: E731
    gate = {r: 0.0 for r in ranks}          # when the next POTRF's inputs are final on rank r
    last_upd = {r: 0.0 for r in ranks}
    panel_ready = {}                        # (rank, k) -> time panel k's tiles are available to rank r
    total_gemm = 0.0
    for b, (c0, c1) in enumerate(blocks):
        for k in range(c0, c1):
            pc = k % Q
            # POTRF(k) on the diagonal owner
            ro = own(k, k)
            dur = m.t_potrf * (m.slow_potrf if overlapped(ro, max(free[(ro, 'panel')], gate[ro])) else 1.0)
            _, t_pot = run(ro, "panel", gate[ro], dur)
            # DBCAST down the owner column, TRSM of the local panel tiles
            t_trsm = {}
            for p in range(P):
                r = (p, pc)
                t_in = t_pot if r == ro else t_pot + (m.msg(tile_b) if P > 1 else 0)
                mine = [i for i in range(k + 1, nt) if i % P == p]
                start = max(free[(r, "panel")], t_in, gate[r])
                dur = m.trsm(len(mine), NB) * (m.slow_trsm if overlapped(r, start) else 1.0)
                _, t_trsm[p] = run(r, "panel", t_in, dur) if mine else (0, max(t_in, free[(r, 'panel')]))
            # PANEL_COMM: row broadcast of each process row's panel tiles, then the column
            # all-gather of the tiles each process column needs as the second operand
            if P * Q > 1:
                t_row = {}
                for p in range(P):
                    cnt = sum(1 for i in range(k + 1, nt) if i % P == p)
                    t_row[p] = t_trsm[p] + (m.msg(cnt * tile_b) if Q > 1 else 0.0)
                for r in ranks:
                    p, q = r
                    sub = sum(1 for i in range(k + 1, nt) if i % Q == q)
                    t_col = max(t_row.values()) + (m.msg(sub * tile_b // P * (P - 1)) if P > 1 else 0.0)
                    t_av = max(t_row[p], t_col)
                    _, t_av = run(r, "panel", t_av, 0.0)
                    panel_ready[(r, k)] = t_av
            else:
                panel_ready[(ro, k)] = t_trsm[0]
            # NEAR(k): the rest of the block on every rank
            for r in ranks:
                p, q = r
                cols = [j for j in range(k + 1, c1) if j % Q == q]
                ntl = sum(1 for j in cols for i in range(j, nt) if i % P == p)
                fl = 2.0 * ntl * NB ** 3
                total_gemm += fl
                _, gate[r] = run(r, "panel", panel_ready[(r, k)], m.gemm(fl, ntl * 4))
        if c1 >= nt:
            break
        n0, n1 = blocks[b + 1]
        kd = (c1 - c0) * NB
        for r in ranks:
            p, q = r

            def tiles(lo, hi):
                return sum(1 for j in range(lo, hi) if j % Q == q for i in range(j, nt) if i % P == p)
            tn, tr = tiles(n0, n1), tiles(n1, nt)
            dep = max(gate[r], last_upd[r])
            fl_n, fl_r = 2.0 * tn * NB * NB * kd, 2.0 * tr * NB * NB * kd
            total_gemm += fl_n + fl_r
            s0, t_next = run(r, "update", dep, m.gemm(fl_n, tn * 4))
            s1, t_rest = run(r, "update", t_next, m.gemm(fl_r, tr * 4))
            busy_upd[r].append((s0, t_rest))
            last_upd[r] = t_rest
            gate[r] = t_next
    end = max(free.values())
    return end


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-N", type=int, default=65536)
    ap.add_argument("--nb", type=int, default=512)
    ap.add_argument("--grids", default="1x1,1x2,2x2,2x4")
    ap.add_argument("--bw", type=float, default=50.0, help="GB/s per broadcast / all-gather")
    ap.add_argument("--lat", type=float, default=20.0, help="us per message")
    ap.add_argument("-D", type=int, default=4)
    ap.add_argument("--calibrate", action="store_true")
    ap.add_argument("--uplo", choices=("L", "U"), default="L",
                    help="U: upper Cholesky on P x Q is lower on Q x P (its panel is a tile row, spread over Q)")
    a = ap.parse_args()
    m = Model(bw=a.bw * 1e9, lat=a.lat * 1e-6)
    fl = lambda n: n ** 3 / 3 + n ** 2 / 2 + n / 6  # noqa: E731
    if a.calibrate:
        for n, t in MEASURED_1GPU.items():
            s = simulate(n, a.nb, 1, 1, m, a.D)
            print(f"1 GPU N={n:6d}: model {s * 1e3:8.1f} ms ({fl(n) / s / 1e12:5.1f} TF/s)   measured "
                  f"{t * 1e3:8.1f} ms ({fl(n) / t / 1e12:5.1f} TF/s)")
    base = None
    for g in a.grids.split(","):
        P, Q = (int(x) for x in g.split("x"))
        s = simulate(a.N, a.nb, *((P, Q) if a.uplo == "L" else (Q, P)), m, a.D)
        tf = fl(a.N) / s / 1e12
        base = base or tf
        print(f"{P}x{Q} N={a.N}: model {s * 1e3:8.1f} ms  {tf:6.1f} TF/s  {100 * tf / (P * Q * PEAK / 1e12):5.1f}% of "
              f"peak  scaling efficiency {100 * tf / (base * P * Q):5.1f}%")


if __name__ == "__main__":
    main()
