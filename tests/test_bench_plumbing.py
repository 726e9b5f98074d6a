"""bench.py multi-rank plumbing: the exact driver command line (torch.distributed.run,
127.0.0.1 rendezvous) on CPU ranks with gloo (--cpu), so the N>1 path of the
headline benchmark is exercised without GPUs."""
import json
import os
import subprocess
import sys

import pytest

from helpers import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("nproc", [2, 4])
def test_bench_multirank_cpu(nproc):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(nproc), "--steps", "2", "--warmup", "1", "--cpu", "-N", "640", "--nb", "64", "--check"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == nproc and out["steps"] == 2 and out["warmup"] == 1
    assert out["check"] is True and out["info"] == 0
    assert out["value"] > 0 and out["higher_is_better"] is True
    for k in ("metric", "unit", "ms_per_step", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in out


def test_bench_spawns_ranks_without_launcher():
    """``bench.py --gpus 4`` with no torch.distributed.run around it starts the 4 ranks itself."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "1", "--warmup", "0",
           "--cpu", "-N", "512", "--nb", "64", "--no-check"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    assert json.loads(lines[0])["n_gpus"] == 4


def test_bench_refuses_missing_gpus():
    """More GPUs requested than visible: non-zero exit and no JSON line (never a mislabelled number)."""
    import torch
    n = torch.cuda.device_count() + 1
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(max(2, n)), "--steps", "1"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert "GPU" in r.stderr


def _race_worker(rank, world, scenario):
    """bench.race_engines on gloo ranks with injected failures: every rank must take the same branch."""
    import importlib.util

    import torch
    import torch.distributed as dist
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)

    def agree(v, op):
        t = torch.tensor([float(v)], dtype=torch.float64)
        dist.all_reduce(t, op=op)
        return float(t.item())
    calls = {"poisoned": 0, "stream": 0}

    def build():
        if scenario == "build_fails" and rank == 1:
            raise RuntimeError("IPC allocation failed")
        return "dtr-handle"

    def run_dtr(tpd, poison=False):
        assert tpd == "dtr-handle"
        calls["poisoned"] += int(poison)
        if scenario == "launch_fails" and rank == world - 1:
            raise RuntimeError("potrf: distributed device task runtime failure (info -1000)")
        # rank 0 slower than the stream engine in "dtr_slow_on_one_rank": the MAX over ranks decides
        return 5.0 if (scenario == "dtr_slow_on_one_rank" and rank == 0) else 1.0

    def check(tpd):
        # a stale cross-GPU read shows up as NaN -> residual failure on that rank only
        return not (scenario == "check_fails" and rank == 1)

    def run_stream():
        calls["stream"] += 1
        return 2.0
    eng, t_d, t_s, _ = bench.race_engines(lambda v: agree(v, dist.ReduceOp.MIN), lambda v: agree(v, dist.ReduceOp.MAX),
                                          build, run_dtr, check, run_stream)
    dist.barrier()   # every collective matched: this returns on every rank
    return eng, calls


@pytest.mark.parametrize("scenario,expect", [("ok", "dtr"), ("build_fails", "stream"), ("launch_fails", "stream"),
                                             ("check_fails", "stream"), ("dtr_slow_on_one_rank", "stream")])
def test_bench_engine_race_falls_back(scenario, expect):
    """The N > 1 warmup race keeps the distributed DTR only if it built, ran and passed the (poisoned-slot)
    residual check on EVERY rank and was faster on the slowest rank; one rank's failure sends all to `stream`."""
    from helpers import run_distributed
    out = run_distributed(_race_worker, 3, scenario)
    engines = {r: v[0] for r, v in out.items()}
    assert set(engines.values()) == {expect}, engines
    for r, (_, calls) in out.items():
        if scenario not in ("build_fails", "launch_fails"):
            assert calls["poisoned"] == 1      # the checked run starts from poisoned receive slots
        assert calls["stream"] == (2 if scenario != "build_fails" else 0)
