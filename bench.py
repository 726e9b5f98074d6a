#!/usr/bin/env python3
"""Headline benchmark: DPOTRF GFLOP/s, N=65536, NB=512, on 1/2/4/8 MI355X.

Metric and config are the ones named in BASELINE.json.  One process per GPU
(``torch.distributed.run --nproc-per-node N``; RCCL over xGMI), 2-D
block-cyclic P x Q grid (8 -> 2x4 as BASELINE.json names it; 2 and 4 -> the whole panel axis:
P x 1 for lower, 1 x Q for upper).  The input is
the reference's SPD test matrix ``dplghe(bump=N, seed=3872)`` (synthetic, LCG
generated on the GPU, bit-identical to the reference generator).

A "step" = one full distributed Cholesky factorisation of the pristine matrix.
Before each step A is restored from a device copy (untimed, as the reference
re-generates A outside its timed region); each of the K timed factorisations
is bracketed by device synchronize + barrier on both sides (the reference's
MPI_Barrier / context_start+wait / MPI_Barrier, tests/common.h:252-277), the
K times are summed, and the max over ranks is reported.  W untimed warm-up
steps come first.  Flops are
FLOPS_DPOTRF(N) = N^3/3 + N^2/2 + N/6 per step (src/flops.h), as in the
reference harness (tests/common.h:136-137, 268-277).  Strong scaling: N is
fixed as the GPU count grows.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

BASELINE_METRIC = "GFLOP/s DPOTRF N=64k NB=512 at 1/2/4/8 MI355X; % of fp64 MFMA peak"
FP64_PEAK_GFLOPS = 78600.0  # per MI355X, datasheet


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn_ranks(n: int, cpu: bool) -> int:
    """``--gpus N`` without a launcher: run this same command under ``torch.distributed.run`` with N
    ranks (127.0.0.1 rendezvous) as a child process; returns its exit status.  Refuses (non-zero)
    when fewer than N GPUs are visible -- a silent 1-GPU number reported as N would be invalid.
    ``torch.cuda.device_count()`` does not initialise the GPU, so no exec/fork hazard here."""
    import subprocess
    if not cpu:
        have = torch.cuda.device_count()
        if have < n:
            print(f"bench.py: --gpus {n} requested but only {have} GPU(s) are visible", file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def race_engines(agree_min, agree_max, build_dtr, run_dtr, check_dtr, run_stream, log=None):
    """The engine race's decision, with every collective injected (agree_min / agree_max: all-reduce of one float
    over the ranks): build the DTR, run it twice (warm, then timed and checked), time the stream engine twice, and
    keep the DTR only if it built, ran and passed the check on EVERY rank and was faster (max over ranks).  A
    failure on one rank -- an exception from build_dtr / run_dtr / check_dtr -- is agreed, never skipped, so
    every rank takes the same branch and no collective is left unmatched.  Returns ("dtr" | "stream", t_dtr,
    t_stream, dtr_handle)."""
    tpd, ok = None, 1.0
    try:
        tpd = build_dtr()
    except Exception as e:   # noqa: BLE001 -- any build failure means: keep the stream engine
        if log:
            log(f"distributed DTR unavailable ({e})")
        ok = 0.0
    if agree_min(ok) < 1:
        return "stream", None, None, None
    # the stream engine runs FIRST: on a GPU shared by several ranks, a DTR run after the stream engine's was measured
    # 4-5x slower than one before it (profiles/r6_bench_race_w4.txt) -- timing the DTR last times it in the state the
    # timed steps will see
    run_stream()
    t_s = run_stream()
    t_d = float("inf")
    try:
        run_dtr(tpd, poison=False)
        t_d = run_dtr(tpd, poison=True)
    except Exception as e:   # noqa: BLE001 -- a drained launch: the taskpool agreed the failure across ranks
        if log:
            log(f"distributed DTR failed ({e})")
        ok = 0.0
    if ok:
        try:
            ok = 1.0 if check_dtr(tpd) else 0.0
        except Exception as e:   # noqa: BLE001
            if log:
                log(f"distributed DTR check failed ({e})")
            ok = 0.0
    ok = agree_min(ok)
    t_d, t_s = agree_max(t_d if ok else 1e30), agree_max(t_s)
    if ok and t_d < t_s:
        return "dtr", t_d, t_s, tpd
    return "stream", (t_d if ok else None), t_s, tpd


def _choose_engine(ctx, uplo, A, A0, tp, args):
    """N > 1: race the distributed device task runtime (models/potrf_dtr_dist.py, push-scheduled, in-kernel
    sends over the IPC-mapped peers; modelled at 75 % of 8-GPU peak at 2x4 64k, profiles/r5_dtr_dist_emulation.txt)
    against the stream engine in the untimed warmup, and keep it only if it builds, factors correctly (residual
    check) and is faster on every rank -- all three agreed across ranks, so every rank picks the same engine.
    The checked run starts from POISONED receive slots and peer W blocks (NaN): a strip read before its bytes
    crossed xGMI fails the check instead of reproducing the previous run's bit-identical values.
    DPLASMA_BENCH_DIST_ENGINE=stream skips the race."""
    import torch.distributed as dist

    import dplasma_amd as dp
    from dplasma_amd.models import potrf_dtr_dist
    if os.environ.get("DPLASMA_BENCH_DIST_ENGINE", "race") == "stream" or args.cpu or \
            not potrf_dtr_dist.supported(ctx, uplo, A):
        return tp, "stream"
    dev = ctx.device

    def agree(v, op):
        t = torch.tensor([float(v)], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=op)
        return float(t.item())

    def timed(t, poison=False):
        A.data.copy_(A0)
        t.info.zero_()
        if poison:
            t.poison()
        ctx.sync()
        ctx.barrier()
        ctx.sync()
        t0 = time.perf_counter()
        t.run(ctx)
        ctx.sync()
        el = time.perf_counter() - t0
        t.complete(ctx)
        return el

    def check(_t):
        A_orig = A.like()
        A_orig.data.copy_(A0)
        good, _ = dp.check_potrf(ctx, uplo, A, A_orig)
        del A_orig
        return good

    engine, t_d, t_s, tpd = race_engines(
        lambda v: agree(v, dist.ReduceOp.MIN), lambda v: agree(v, dist.ReduceOp.MAX),
        lambda: potrf_dtr_dist.potrf_dtr_dist_New(ctx, uplo, A), timed, check, lambda: timed(tp),
        log=lambda m: print(f"rank {ctx.rank}: {m}", file=sys.stderr))
    if ctx.rank == 0:
        print(f"bench: warmup race -- distributed DTR {'%.1f ms' % (t_d * 1e3) if t_d else 'not usable'}, "
              f"stream engine {'%.1f ms' % (t_s * 1e3) if t_s else '-'} (checked run from poisoned receive slots)",
              file=sys.stderr)
    if engine == "dtr":
        return tpd, "dtr"
    potrf_dtr_dist.release_all()
    return tp, "stream"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("-N", "--N", type=int, default=65536)
    ap.add_argument("--nb", type=int, default=512)
    ap.add_argument("-P", type=int, default=None)
    ap.add_argument("--uplo", choices=("L", "U"), default="L",
                    help="triangle factored (the reference's testing_zpotrf.c defaults to Upper)")
    ap.add_argument("--no-check", dest="check", action="store_false",
                    help="skip the (untimed, default-on) residual check of the last factorisation")
    ap.add_argument("--check", dest="check", action="store_true", help="(default) verify the last factorisation")
    ap.add_argument("--trace", default=None, help="write a Chrome trace of one step to this file")
    ap.add_argument("--cpu", action="store_true",
                    help="dry run of the same multi-rank path on CPU ranks (gloo) -- plumbing tests only")
    args = ap.parse_args()

    if args.gpus < 1:
        sys.exit(f"bench.py: --gpus must be >= 1 (got {args.gpus})")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: start one rank per GPU ourselves (a child torch.distributed.run, before any GPU
        # call in this process) and exit with its status
        sys.exit(_spawn_ranks(args.gpus, args.cpu))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)")
    if world > 1:
        import datetime
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        local = int(os.environ.get("LOCAL_RANK", "0"))
        # a hung exchange ends the run (non-zero exit) instead of blocking until the driver's limit
        pg_timeout = datetime.timedelta(seconds=int(os.environ.get("DPLASMA_PG_TIMEOUT", "300")))
        if args.cpu:
            dist.init_process_group("gloo", timeout=pg_timeout)
        elif os.environ.get("DPLASMA_DIST_BACKEND") == "gloo":
            # rehearsal of the multi-rank GPU path on fewer GPUs than ranks (gloo moves GPU tensors
            # through the host); ranks share devices round-robin
            local %= torch.cuda.device_count()
            torch.cuda.set_device(local)
            dist.init_process_group("gloo", timeout=pg_timeout)
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=pg_timeout)
    import dplasma_amd as dp

    P = args.P
    if P is None:
        # The panel of lower Cholesky is a tile column (spread over the P process rows), that of upper a
        # tile row (spread over the Q columns).  A grid whose panel axis holds every rank (P x 1 for
        # lower, 1 x Q for upper) splits the panel TRSM over all of them and moves the panel by one
        # all-gather instead of a broadcast to ranks that own none of it -- tools/sim_potrf.py: 88 vs 75 %
        # on 2 GPUs, 59 vs 54 % on 4.  8 GPUs keep the grid BASELINE.json names (2 x 4).
        if world == 8:
            P = 2
        elif world in (2, 4):
            P = world if args.uplo == "L" else 1
        else:
            P = None
    ctx = dp.init(P=P, device="cpu") if args.cpu else dp.init(P=P)
    rank = ctx.rank
    N, NB = args.N, args.nb
    uplo = dp.dplasmaLower if args.uplo == "L" else dp.dplasmaUpper
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N, name="A", uplo=uplo)
    dp.dplghe(ctx, float(N), uplo, A, 3872)
    A0 = A.data.clone()
    ctx.sync()
    t0 = time.perf_counter()
    tp = dp.dpotrf_New(ctx, uplo, A)
    t_enq = time.perf_counter() - t0
    flops = tp.flops
    engine = "dtr" if getattr(tp, "dtr_plan", None) is not None else "stream"
    if world > 1:
        tp, engine = _choose_engine(ctx, uplo, A, A0, tp, args)

    def step():
        A.data.copy_(A0)
        tp.info.zero_()
        tp.run(ctx)

    for _ in range(args.warmup):
        step()
    tp.complete(ctx)
    ctx.barrier()
    ctx.sync()
    total = 0.0
    # DPLASMA_BENCH_STEPLOG=1: every rank prints each timed step's time (stderr) -- the per-step view behind the max
    steplog = os.environ.get("DPLASMA_BENCH_STEPLOG") == "1"
    for si in range(args.steps):
        A.data.copy_(A0)
        tp.info.zero_()
        ctx.sync()
        ctx.barrier()
        ctx.sync()
        t0 = time.perf_counter()
        tp.run(ctx)
        ctx.sync()
        ctx.barrier()
        ctx.sync()
        dt = time.perf_counter() - t0
        total += dt
        if steplog:
            print(f"bench: rank {rank} step {si}: {dt * 1e3:.1f} ms", file=sys.stderr)
    info = tp.complete(ctx)
    el = torch.tensor([total], dtype=torch.float64, device=ctx.device)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    ms = elapsed / args.steps * 1e3
    gflops = flops * args.steps / elapsed / 1e9
    ok, res = None, None
    if args.check:
        # untimed: verify the last timed factorisation (reference check_zpotrf, src/dplasma_zcheck.c)
        tc = time.perf_counter()
        A_orig = A.like()
        A_orig.data.copy_(A0)
        del A0
        ok, res = dp.check_potrf(ctx, uplo, A, A_orig, verbose=(rank == 0))
        t_check = time.perf_counter() - tc
        del A_orig
    if rank == 0:
        print(f"[****] TIME(s) {ms / 1e3:12.5f} : dpotrf PxQxg= {ctx.P:3d} {ctx.Q:<3d} 1 NB= {NB:4d} N= {N:7d} : "
              f"{gflops / world:14f} gflops/gpu - ENQ {t_enq:.3f} info={info}", file=sys.stderr)
        out = {
            "metric": BASELINE_METRIC,
            "value": round(gflops, 2),
            "unit": "GFLOP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "fp64",
            "data": "synthetic (dplghe SPD, bump=N, seed=3872; random-init, LCG generated on GPU)",
            "pct_fp64_peak": round(100.0 * gflops / (FP64_PEAK_GFLOPS * world), 2),
            "info": info,
            "check": ok,
            "residual": res,
            "check_s": round(t_check, 2) if args.check else None,
            "enq_s": round(t_enq, 3),
            "engine": engine,
            "config": {"model": f"dpotrf ({'lower' if args.uplo == 'L' else 'upper'}, 2D block-cyclic tiles)", "N": N, "NB": NB, "global_batch": 1,
                       "seq_len": N, "parallelism": f"{ctx.P}x{ctx.Q} block-cyclic (one rank per GPU)"},
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
