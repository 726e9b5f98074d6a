#!/usr/bin/env python3
"""Rank replay of the distributed Cholesky on ONE GPU.

Compiles the exact ``potrf_New`` program of rank r of a P x Q grid (its local tiles, its panel
slabs, its tasks and streams -- models/potrf_dist.py) and runs it on the one visible GPU with the
transport replaced by a timing model (``parallel.comm.set_backend``):

* every grouped send/recv batch becomes a busy-wait kernel (``dpl_delay``, ``--comm-wg`` workgroups,
  like the RCCL kernel it stands for) on a high-priority stream per communicator -- batches of one
  communicator serialise, as on RCCL -- lasting ``lat + max_peer_bytes / bw`` (one xGMI link per
  peer pair);
* a batch that only receives data produced remotely first runs a proxy of the producer's
  critical-path kernel on this GPU (the diagonal-tile POTRF for the diagonal triangle, the panel
  TRSM of the root's tile count for a panel piece), so the arrival time includes the producer's
  chain AND its slowdown beside a bulk update (the proxy competes with this rank's bulk GEMM the way
  the producer's kernel competes with its own);
* the received bytes are not moved: the numbers in the slabs are stale, which does not change the
  kernels' run time (the tile kernels are data-independent; info is ignored).

It is an optimistic-symmetric model: remote producers are assumed to reach panel k when this rank
does.  Per-rank span = wall time of ``tp.run`` + synchronize (the reference's timed region).

usage: python tools/replay_potrf.py -N 65536 --nb 512 --grid 2x4 --ranks all --steps 2
       [--bw 50] [--lat 15] [--uplo L]   (DPLASMA_POTRF_* knobs via the environment)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import dplasma_amd as dp  # noqa: E402
from dplasma_amd.ops import _lib  # noqa: E402
from dplasma_amd.ops import tile_ops as ops  # noqa: E402
from dplasma_amd.parallel import comm  # noqa: E402


class ReplayBackend:
    def __init__(self, dev, bw_gbs: float, lat_us: float, nwg: int, proxies: bool = True):
        self.dev = torch.device(dev)
        self.bw = bw_gbs * 1e3        # bytes per us
        self.lat = lat_us
        self.nwg = nwg
        self.proxies = proxies
        self.streams = {}
        if self.dev.type == "cuda":
            lo, hi = torch.cuda.Stream.priority_range()
            self.hi = hi
            self.remote = torch.cuda.Stream(device=dev, priority=hi)
            self.remote_potrf = self.remote_trsm = self.remote   # CU-partitioned runs: the rank's own streams
            self.lib = _lib.load()
        self.stats = {"batches": 0, "bytes": 0, "us": 0.0, "proxy_potrf": 0, "proxy_trsm": 0}
        self._scratch = {}

    def _stream(self, group):
        key = id(group) if group is not None else 0
        s = self.streams.get(key)
        if s is None:
            s = self.streams[key] = torch.cuda.Stream(device=self.dev, priority=self.hi)
        return s

    # -- proxies of the producer's kernels (identity data: always SPD, never NaN)
    def _potrf_proxy(self, kb):
        key = ("potrf", kb)
        sc = self._scratch.get(key)
        if sc is None:
            t = torch.eye(kb, dtype=torch.float64, device=self.dev).t().contiguous().view(-1)
            sc = self._scratch[key] = (t, torch.zeros(1, dtype=torch.int32, device=self.dev),
                                       torch.empty(ops.rb_zbuf_size(), dtype=torch.float64, device=self.dev))
        t, inf, z = sc
        t.view(kb, kb).copy_(torch.eye(kb, dtype=torch.float64, device=self.dev))
        ops.potrf_tile(dp.dplasmaLower, t, 0, kb, kb, inf, 0, zbuf=z)
        self.stats["proxy_potrf"] += 1

    def _trsm_proxy(self, cnt, kb):
        if cnt <= 0:
            return
        key = ("trsm", cnt, kb)
        sc = self._scratch.get(key)
        if sc is None:
            L = torch.eye(kb, dtype=torch.float64, device=self.dev).contiguous().view(-1)
            z = torch.empty(ops.rb_zbuf_size(), dtype=torch.float64, device=self.dev)
            ops.trsm_rb_prep(dp.dplasmaLower, kb, L, 0, kb, z)
            B = torch.zeros(cnt * kb * kb, dtype=torch.float64, device=self.dev)
            # cnt tiles stacked as one (cnt*kb) x kb column block, ld = cnt*kb
            pan = ops.RbPanel(dp.dplasmaLower, [(i * kb, kb) for i in range(cnt)], cnt * kb)
            sc = self._scratch[key] = (L, z, B, pan)
        L, z, B, pan = sc
        ops.trsm_rb(dp.dplasmaLower, kb, L, 0, kb, z, pan, B, cnt * kb)
        self.stats["proxy_trsm"] += 1

    def start_p2p(self, sends, recvs, group, hint):
        if self.dev.type != "cuda":   # CPU dry run (tests): the program's control flow only
            self.stats["batches"] += 1
            return comm.Pending((), device=False)
        cur = torch.cuda.current_stream(self.dev)
        gs = self._stream(group)
        ev = torch.cuda.Event()
        ev.record(cur)
        # critical link: per peer the larger direction (full-duplex xGMI links)
        out_b, in_b = {}, {}
        for t, p in sends:
            out_b[p] = out_b.get(p, 0) + t.numel() * t.element_size()
        for t, p in recvs:
            in_b[p] = in_b.get(p, 0) + t.numel() * t.element_size()
        per_peer = {p: max(out_b.get(p, 0), in_b.get(p, 0)) for p in set(out_b) | set(in_b)}
        if self.proxies and recvs and not sends and hint is not None:
            rs = self.remote_potrf if hint[0] == "potrf" else self.remote_trsm
            rs.wait_event(ev)
            with torch.cuda.stream(rs):
                if hint[0] == "potrf":
                    self._potrf_proxy(hint[1])
                elif hint[0] == "trsm":
                    self._trsm_proxy(hint[1], hint[2])
            ev = torch.cuda.Event()
            ev.record(rs)
        gs.wait_event(ev)
        us = self.lat + max(per_peer.values()) / self.bw
        _lib.check(self.lib.dpl_delay(float(us), self.nwg, gs.cuda_stream), "delay")
        end = torch.cuda.Event()
        end.record(gs)
        self.stats["batches"] += 1
        self.stats["bytes"] += sum(t.numel() * t.element_size() for t, _ in recvs)
        self.stats["us"] += us
        return comm.Pending((), device=True, meta=end)

    def finish(self, p):
        if p.meta is not None:
            torch.cuda.current_stream(self.dev).wait_event(p.meta)

    def sync(self, kind, nbytes, group):
        """A blocking collective / point-to-point exchange (bcast, allgather, allreduce, p2p): one delay
        kernel of lat + critical-link bytes / bw on the group's communication stream, waited for by
        the current stream (the data is not moved)."""
        self.stats["sync_" + kind] = self.stats.get("sync_" + kind, 0) + 1
        if self.dev.type != "cuda":
            return
        cur = torch.cuda.current_stream(self.dev)
        gs = self._stream(group)
        ev = torch.cuda.Event()
        ev.record(cur)
        gs.wait_event(ev)
        us = self.lat + nbytes / self.bw
        _lib.check(self.lib.dpl_delay(float(us), self.nwg, gs.cuda_stream), "delay")
        end = torch.cuda.Event()
        end.record(gs)
        cur.wait_event(end)
        self.stats["us"] += us


def fake_rank_context(base, P, Q, rank):
    """The one-GPU context dressed as rank ``rank`` of a P x Q grid (no process group)."""
    c = object.__new__(type(base))
    c.__dict__.update(base.__dict__)
    c.distributed, c.world, c.rank = True, P * Q, rank
    c.P, c.Q = P, Q
    c.myrow, c.mycol = rank // Q, rank % Q
    c.row_group = c.col_group = None
    c.urgent_group = "urgent"
    c.bulk_groups = [f"bulk{i}" for i in range(int(os.environ.get("DPLASMA_BULK_GROUPS", "2")))]
    c._queue = []
    return c


def replay_rank(base, P, Q, rank, N, NB, uplo, steps, backend):
    ctx = fake_rank_context(base, P, Q, rank)
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N, name="A", uplo=uplo)
    # a well-conditioned SPD-looking local share (values do not matter for the timing)
    dp.dplghe(ctx, float(N), uplo, A, 3872)
    A0 = A.data.clone()
    t0 = time.perf_counter()
    tp = dp.dpotrf_New(ctx, uplo, A)
    t_enq = time.perf_counter() - t0
    times = []
    gpu = ctx.is_gpu
    for s in range(steps + 1):
        A.data.copy_(A0)
        if gpu:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        tp.run(ctx)
        if gpu:
            torch.cuda.synchronize()
        if s > 0:             # the first run is a warm-up
            times.append(time.perf_counter() - t0)
    del A, A0, tp
    if gpu:
        torch.cuda.empty_cache()
    return min(times), t_enq


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-N", type=int, default=65536)
    ap.add_argument("--nb", type=int, default=512)
    ap.add_argument("--grid", default="2x4")
    ap.add_argument("--ranks", default="all", help="'all' or a comma list")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--bw", type=float, default=50.0, help="GB/s per peer link (one direction)")
    ap.add_argument("--lat", type=float, default=15.0, help="us per batch")
    ap.add_argument("--comm-wg", type=int, default=4)
    ap.add_argument("--no-proxy", action="store_true")
    ap.add_argument("--uplo", choices=("L", "U"), default="L")
    args = ap.parse_args()
    P, Q = map(int, args.grid.lower().split("x"))
    uplo = dp.dplasmaLower if args.uplo == "L" else dp.dplasmaUpper
    base = dp.init(device="cuda:0")
    be = ReplayBackend(base.device, args.bw, args.lat, args.comm_wg, proxies=not args.no_proxy)
    comm.set_backend(be)
    tile_cus = int(os.environ.get("DPLASMA_POTRF_TILE_CUS", "0"))
    if tile_cus > 0:
        # the remote producers run their tile kernels on their own partition, as this rank does
        s_tile, s_chain, _ = base.partition_streams(tile_cus)
        be.remote_potrf, be.remote_trsm = base.streams[s_tile], base.streams[s_chain]
    ranks = range(P * Q) if args.ranks == "all" else [int(x) for x in args.ranks.split(",")]
    fl = dp.flops_of("d", "potrf", args.N) if hasattr(dp, "flops_of") else None
    if fl is None:
        from dplasma_amd.utils.flops import flops
        fl = flops("d", "potrf", args.N)
    knobs = {k: v for k, v in os.environ.items() if k.startswith("DPLASMA_")}
    res = {}
    for r in ranks:
        t, enq = replay_rank(base, P, Q, r, args.N, args.nb, uplo, args.steps, be)
        res[r] = t
        print(f"rank {r} ({r // Q},{r % Q}): {t * 1e3:9.2f} ms   enq {enq:.2f} s", flush=True)
    worst = max(res.values())
    ideal = fl / (78.6e12 * P * Q)
    out = {"N": args.N, "NB": args.nb, "grid": f"{P}x{Q}", "uplo": args.uplo, "bw_GBs": args.bw, "lat_us": args.lat,
           "worst_ms": round(worst * 1e3, 2), "ideal_ms": round(ideal * 1e3, 2),
           "pct_peak": round(100 * ideal / worst, 1), "tflops_job": round(fl / worst / 1e12, 1),
           "per_rank_ms": {str(k): round(v * 1e3, 2) for k, v in res.items()}, "knobs": knobs,
           "comm": {k: (round(v, 1) if isinstance(v, float) else v) for k, v in be.stats.items()}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
