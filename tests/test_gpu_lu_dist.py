"""Distributed-pivoting LU panel on the GPU (ops.lu_dist_ops / csrc/kernels/lu_dist.hip): two ranks
share one MI355X and exchange every column's pivot candidates through IPC-mapped device buffers inside
the persistent panel kernel.  Pivots must be identical to the one-process factorisation on the same
GPU (tools/gpu/lu_dist_rehearsal.py does the check and prints SUCCESS)."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _run(world, N, NB, extra_env=None, timeout=240, P=None):
    env = dict(os.environ, DPLASMA_DIST_BACKEND="gloo", PYTHONUNBUFFERED="1")
    env.update(extra_env or {})
    port = 29600 + world + (N // NB) % 50
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(ROOT / "tools/gpu/lu_dist_rehearsal.py"),
           str(N), str(NB), str(P or world)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    out = r.stdout + r.stderr
    return r.returncode, out


@pytest.mark.gpu
@pytest.mark.parametrize("world,N,NB", [(2, 2048, 256), (2, 3000, 256), (4, 4096, 512)])
def test_lu_dist_ipc(world, N, NB):
    rc, out = _run(world, N, NB)
    print(out[-3000:])
    assert rc == 0, out[-3000:]
    assert out.count("SUCCESS") == world and "exchange=ipc" in out


@pytest.mark.gpu
def test_lu_dist_host_exchange_on_gpu():
    """The transport-independent path (one all-gather per column) on GPU tensors: same pivots."""
    rc, out = _run(2, 1024, 128, {"DPLASMA_LU_XCHG": "host"})
    assert rc == 0, out[-3000:]
    assert out.count("SUCCESS") == 2 and "exchange=host" in out


@pytest.mark.gpu
@pytest.mark.parametrize("panel", ["gather", "dist"])
def test_lu_grid_2x4_rehearsal(panel):
    """The whole P x Q program on a 2 x 4 grid of eight processes sharing the GPU: point-to-point interchanges of the
    rows crossing process rows, chunked trailing exchanges, look-ahead, the panel rows' own LSEND buffers (the shared
    receive buffer gave intermittently wrong factors).  Pivots and factors equal one process."""
    rc, out = _run(8, 4096, 256, {"DPLASMA_LU_PANEL": panel}, timeout=400, P=2)
    assert rc == 0, out[-3000:]
    assert out.count("SUCCESS") == 8 and "2x4" in out


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{"DPLASMA_LU_LOOKAHEAD": "0"}, {"DPLASMA_LU_XROWS": "allreduce"}])
def test_lu_grid_2x4_gather_modes(env):
    """Gather panels without look-ahead (the panel column sends the pivots inline) and with the summed row exchange
    (the panel slots still travel point to point): both were broken before round 6's fixes."""
    rc, out = _run(8, 4096, 256, dict(env, DPLASMA_LU_PANEL="gather"), timeout=400, P=2)
    assert rc == 0, out[-3000:]
    assert out.count("SUCCESS") == 8
