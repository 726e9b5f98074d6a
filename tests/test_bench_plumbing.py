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
