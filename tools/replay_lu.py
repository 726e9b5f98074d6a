#!/usr/bin/env python3
"""Rank replay of the distributed partial-pivoting LU (getrf_ptgpanel, BASELINE config 5) on ONE GPU.

Builds the exact ``getrf_ptgpanel_New`` program of rank r of a P x Q grid (models/lu.py _GetrfDev: its
local tiles, panel buffers, row moves, U broadcasts, trailing GEMMs) and runs it on the visible GPU with
the transport replaced by the timing model of tools/replay_potrf.py (every collective / point-to-point
exchange = one busy-wait kernel of lat + bytes / bw on a communication stream, no data moved).  The
distributed panel kernel (csrc/kernels/lu_dist.hip) runs on this rank's rows plus the diagonal replica
with a one-rank exchange group, and each column's cross-rank hand-off -- IPC stores over xGMI on a real
grid -- is modelled as ``--xlat`` + ``--xgmi`` microseconds per column on the panel's stream: ``--xlat`` is the
MEASURED cost of a real peer (tools/gpu/lu_xlat_probe.py: two emulated ranks on the two CU halves of one GPU
exchanging through memory, minus one rank alone -- profiles/r6_lu_xlat_probe.txt), ``--xgmi`` the extra one-way
latency of an xGMI hop over an on-package one (an assumption, reported with the result).

Communicators are modelled separately (one delay stream each): the row / column groups of the panel and
diagonal-tile broadcasts, the urgent communicator of the next column's interchanges and U block, the bulk ones of
the rest of the trailing columns and of the deferred left-column interchanges (models/lu.py _xswap).

usage: python tools/replay_lu.py -N 65536 --nb 512 --grid 2x4 [--ranks all] [--steps 1] [--bw 50]
       [--lat 15] [--xlat 2.4] [--xgmi 2]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# one hardware queue per modelled link stream: with HIP's default of 4 queues per process the delay streams of
# the five communicators (and the program's panel / update / exchange / side streams) share queues, which
# serialises transfers that run on different links (--hw-queues, default 16; set before HIP starts)
if "--hw-queues" in sys.argv:
    os.environ["GPU_MAX_HW_QUEUES"] = sys.argv[sys.argv.index("--hw-queues") + 1]
else:
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import dplasma_amd as dp  # noqa: E402
from dplasma_amd.ops import lu_dist_ops  # noqa: E402
from dplasma_amd.parallel import comm  # noqa: E402
from replay_potrf import ReplayBackend, fake_rank_context  # noqa: E402


class ReplayXchg:
    """A one-rank exchange group for the distributed panel kernel (its own slot is the only peer), with
    the per-column cross-rank hand-off modelled as a delay (lu_dist_ops.PanelLU.run)."""

    def __init__(self, kbw, dtype, device, xlat_us):
        from dplasma_amd.ops import _lib
        lib = _lib.load()
        self.group, self.me, self.P = None, 0, 1
        self.slot_bytes = int(lib.dpl_lu_dist_slot_bytes(_lib.prec_code(dtype), kbw))
        self.buf = torch.zeros(2 * self.slot_bytes // 8 + 8, dtype=torch.float64, device=device)
        self.peers = torch.tensor([self.buf.data_ptr()], dtype=torch.int64, device=device)
        self.epoch = 1
        self.ok = True
        self.model_us_per_col = xlat_us

    def close(self):
        pass


def true_pivots(base, N, NB):
    """The pivots of the whole factorisation, from a one-process getrf_ptgpanel of the same matrix
    (plrnt seed 3872, identical for every distribution): what each panel's broadcast delivers on the grid."""
    A = dp.block_cyclic(base, torch.float64, NB, NB, N, N, name="A")
    dp.plrnt(base, A, 3872)
    IP = dp.ptgpanel_ipiv_descriptor(base, A)
    tp = dp.getrf_ptgpanel_New(base, A, IP)
    info = tp.execute(base)
    ipiv = tp.ipiv_all.clone()            # global, 1-based
    del A, IP, tp
    torch.cuda.empty_cache()
    return ipiv, info


def _delivered_pivots_panel(orig, ipiv):
    """The replay moves no data, so the pivots a rank computes or receives for panel k are not the grid's
    (a rank outside the panel's process column keeps an earlier panel's vector; a rank inside searched its
    own rows only).  The modelled broadcast instead DELIVERS the true pivots of panel k (from a one-process
    factorisation of the same matrix, ``true_pivots``), as the root's broadcast does on the grid: the row
    moves then carry the real interchange pattern and always stay inside the panel's rows."""
    def panel(self, k):
        orig(self, k)
        st = self.plan[k]
        kmin, r0 = st["kmin"], st["r0"]
        if kmin > 0 and self.pivot:
            self.piv_dev[:kmin] = ipiv[r0:r0 + kmin] - (r0 + 1)
    return panel


def replay_rank(base, P, Q, rank, N, NB, steps, xlat, ipiv):
    from dplasma_amd.models import lu as lu_mod
    ctx = fake_rank_context(base, P, Q, rank)
    ctx.row_group, ctx.col_group = "row", "col"      # one modelled link stream per communicator
    orig = lu_dist_ops.panel_xchg
    orig_panel = lu_mod._GetrfDev.panel
    lu_dist_ops.panel_xchg = lambda group, me, P_, kbw, dtype, device, max_rows=0: ReplayXchg(kbw, dtype, device, xlat)
    lu_mod._GetrfDev.panel = _delivered_pivots_panel(orig_panel, ipiv)
    try:
        A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N, name="A")
        dp.plrnt(ctx, A, 3872)
        A0 = A.data.clone()
        IP = dp.ptgpanel_ipiv_descriptor(ctx, A)
        t0 = time.perf_counter()
        tp = dp.getrf_ptgpanel_New(ctx, A, IP)
        enq = time.perf_counter() - t0
        times = []
        for s in range(steps + 1):
            A.data.copy_(A0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tp.run(ctx)
            torch.cuda.synchronize()
            if s > 0:
                times.append(time.perf_counter() - t0)
        del A, A0, tp
        torch.cuda.empty_cache()
    finally:
        lu_dist_ops.panel_xchg = orig
        lu_mod._GetrfDev.panel = orig_panel
    return min(times), enq


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-N", type=int, default=65536)
    ap.add_argument("--nb", type=int, default=512)
    ap.add_argument("--grid", default="2x4")
    ap.add_argument("--ranks", default="all")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--bw", type=float, default=50.0)
    ap.add_argument("--lat", type=float, default=15.0)
    ap.add_argument("--comm-wg", type=int, default=4)
    ap.add_argument("--xlat", type=float, default=6.0, help="us per panel column (cross-rank pivot hand-off, measured)")
    ap.add_argument("--xgmi", type=float, default=0.0, help="extra us per panel column for the xGMI hop (assumed)")
    ap.add_argument("--hw-queues", type=int, default=16, help="GPU_MAX_HW_QUEUES for this process")
    args = ap.parse_args()
    P, Q = map(int, args.grid.lower().split("x"))
    base = dp.init(device="cuda:0")
    t0 = time.perf_counter()
    ipiv, info0 = true_pivots(base, args.N, args.nb)
    print(f"true pivots: one-process getrf_ptgpanel N={args.N} info={info0} ({time.perf_counter() - t0:.1f} s)",
          flush=True)
    be = ReplayBackend(base.device, args.bw, args.lat, args.comm_wg, proxies=False)
    comm.set_backend(be)
    ranks = range(P * Q) if args.ranks == "all" else [int(x) for x in args.ranks.split(",")]
    from dplasma_amd.utils.flops import flops
    fl = flops("d", "getrf", args.N, args.N)
    res = {}
    for r in ranks:
        t, enq = replay_rank(base, P, Q, r, args.N, args.nb, args.steps, args.xlat + args.xgmi, ipiv)
        res[r] = t
        print(f"rank {r} ({r // Q},{r % Q}): {t * 1e3:9.2f} ms   enq {enq:.2f} s", flush=True)
    worst = max(res.values())
    ideal = fl / (78.6e12 * P * Q)
    print(json.dumps({"op": "getrf_ptgpanel", "N": args.N, "NB": args.nb, "grid": f"{P}x{Q}", "bw_GBs": args.bw,
                      "lat_us": args.lat, "xlat_us_per_col": args.xlat, "xgmi_us_per_col": args.xgmi, "worst_ms": round(worst * 1e3, 2),
                      "ideal_ms": round(ideal * 1e3, 2), "pct_peak": round(100 * ideal / worst, 1),
                      "tflops_job": round(fl / worst / 1e12, 1),
                      "per_rank_ms": {str(k): round(v * 1e3, 2) for k, v in res.items()},
                      "knobs": {k: v for k, v in os.environ.items() if k.startswith("DPLASMA_") or k == "GPU_MAX_HW_QUEUES"},
                      "comm": {k: (round(v, 1) if isinstance(v, float) else v) for k, v in be.stats.items()}}),
          flush=True)


if __name__ == "__main__":
    main()
