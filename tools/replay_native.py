#!/usr/bin/env python3
"""Rank replay of the NATIVE (interpreter-free) distributed Cholesky on one GPU.

Each rank r of a P x Q grid is built with ``dplasma_init_native_dist(dev, r, P*Q, P, ...)`` under
``DPLASMA_NATIVE_TRANSPORT=replay`` (capi/native_comm.cpp ReplayComm): the rank's exact stream program
(capi/native_dist.cpp nat_dist_potrf -- its local tiles, panel slabs, tasks and streams) runs on the one
visible GPU, every exchange replaced by a busy-wait kernel of lat + busiest-link bytes / bw on the
communication stream (no data moves).  Same model as tools/replay_potrf.py --no-proxy, so the two
engines' schedules compare directly.  The C library is driven through ctypes; the engine itself
never touches Python.

usage: python tools/replay_native.py -N 65536 --nb 512 --grid 2x4 [--ranks all] [--steps 2]
       [--bw 50] [--lat 15] [--comm-wg 4]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-N", type=int, default=65536)
    ap.add_argument("--nb", type=int, default=512)
    ap.add_argument("--grid", default="2x4")
    ap.add_argument("--ranks", default="all")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--bw", type=float, default=50.0)
    ap.add_argument("--lat", type=float, default=15.0)
    ap.add_argument("--comm-wg", type=int, default=4)
    ap.add_argument("--uplo", choices=("L", "U"), default="L")
    args = ap.parse_args()
    os.environ["DPLASMA_NATIVE_TRANSPORT"] = "replay"
    os.environ["DPLASMA_REPLAY_BW"] = str(args.bw)
    os.environ["DPLASMA_REPLAY_LAT"] = str(args.lat)
    os.environ["DPLASMA_REPLAY_WG"] = str(args.comm_wg)
    lib = ctypes.CDLL(os.path.join(ROOT, "dplasma_amd", "lib", "libdplasma.so"))
    vp = ctypes.c_void_p
    lib.dplasma_init_native_dist.restype = vp
    lib.dplasma_init_native_dist.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_char_p]
    lib.dplasma_desc_block_cyclic.restype = vp
    lib.dplasma_desc_block_cyclic.argtypes = [vp] + [ctypes.c_int] * 8
    lib.dplasma_dplghe.argtypes = [vp, ctypes.c_double, ctypes.c_int, vp, ctypes.c_ulonglong]
    lib.dplasma_dpotrf.argtypes = [vp, ctypes.c_int, vp]
    lib.dplasma_desc_destroy.argtypes = [vp]
    lib.dplasma_fini.argtypes = [vp]
    lib.dplasma_last_error.restype = ctypes.c_char_p
    P, Q = map(int, args.grid.lower().split("x"))
    uplo = 122 if args.uplo == "L" else 121
    ranks = range(P * Q) if args.ranks == "all" else [int(x) for x in args.ranks.split(",")]
    fl = args.N ** 3 / 3.0
    res = {}
    for r in ranks:
        ctx = lib.dplasma_init_native_dist(0, r, P * Q, P, None)
        if not ctx:
            raise SystemExit(f"init: {lib.dplasma_last_error().decode()}")
        A = lib.dplasma_desc_block_cyclic(ctx, 3, args.nb, args.nb, args.N, args.N, 0, 0, 123)
        if not A:
            raise SystemExit(f"desc: {lib.dplasma_last_error().decode()}")
        times = []
        for s in range(args.steps + 1):
            lib.dplasma_dplghe(ctx, float(args.N), uplo, A, 3872)
            t0 = time.perf_counter()
            info = lib.dplasma_dpotrf(ctx, uplo, A)   # blocking: the program has drained when it returns
            t = time.perf_counter() - t0
            if info < 0:
                raise SystemExit(f"potrf rank {r}: {info} {lib.dplasma_last_error().decode()}")
            if s > 0:
                times.append(t)
        res[r] = min(times)
        print(f"rank {r} ({r // Q},{r % Q}): {res[r] * 1e3:9.2f} ms", flush=True)
        lib.dplasma_desc_destroy(A)
        lib.dplasma_fini(ctx)
    worst = max(res.values())
    ideal = fl / (78.6e12 * P * Q)
    print(json.dumps({"engine": "native", "N": args.N, "NB": args.nb, "grid": f"{P}x{Q}", "bw_GBs": args.bw,
                      "lat_us": args.lat, "worst_ms": round(worst * 1e3, 2), "ideal_ms": round(ideal * 1e3, 2),
                      "pct_peak": round(100 * ideal / worst, 1),
                      "per_rank_ms": {str(k): round(v * 1e3, 2) for k, v in res.items()},
                      "knobs": {k: v for k, v in os.environ.items() if k.startswith("DPLASMA_")}}), flush=True)


if __name__ == "__main__":
    sys.exit(main())
