"""Loopback rehearsal of the distributed transport (``DPLASMA_LOOPBACK=1`` on a world-1 group).

Every algorithm here plans its exchanges as on a real grid, with the rank itself as the peer of
every would-be remote tile edge (parallel.comm module docstring).  The results must equal the
exchange-free single-process path, and the transport must actually have moved tiles:

* POTRF (models/potrf_dist.py: the urgent / bulk point-to-point batches, diagonal-triangle
  send + receive-side unpack / PREP),
* SUMMA GEMM (parallel/exchange.py all-to-all),
* TRSM (a TileProgram: parallel/p2p.Transport),
* incremental-pivoting LU (a tile DAG: fetches into the slot arena and write-backs).

CPU (gloo, which cannot connect a rank to itself): the self pairs complete as local copies, which
checks the planning.  GPU (``-m gpu``): world-1 NCCL group -- real RCCL self send / receive, the
branches a multi-GPU run takes (VERDICT r3 "every RCCL code path is unexecuted").
"""
import os

import pytest
import torch

from helpers import run_distributed

N, NB = 160, 32


def _algos(ctx, dev):
    import dplasma_amd as dp
    out = {}
    # POTRF
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plghe(ctx, float(N), dp.dplasmaLower, A, 3872)
    tp = dp.potrf_New(ctx, dp.dplasmaLower, A)
    info = tp.execute(ctx)
    out["potrf"] = (info, A.to_dense_local().tril().cpu())
    out["potrf_tasks"] = sorted({t.name.split("(")[0] for t in tp.tasks})
    # SUMMA GEMM
    Ag = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N - NB)
    Bg = dp.block_cyclic(ctx, torch.float64, NB, NB, N - NB, N)
    Cg = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plrnt(ctx, Ag, 3872)
    dp.plrnt(ctx, Bg, 4674)
    dp.plrnt(ctx, Cg, 2873)
    tp = dp.gemm_New(ctx, dp.dplasmaNoTrans, dp.dplasmaNoTrans, 0.51, Ag, Bg, -0.42, Cg)
    out["gemm_tasks"] = sorted({t.name.split("(")[0] for t in tp.tasks})
    tp.execute(ctx)
    out["gemm"] = Cg.to_dense_local().cpu()
    # TRSM (TileProgram)
    T = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plghe(ctx, float(N), dp.dplasmaLower, T, 11)
    X = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N // 2)
    dp.plrnt(ctx, X, 12)
    tp = dp.trsm_New(ctx, dp.dplasmaLeft, dp.dplasmaLower, dp.dplasmaNoTrans, dp.dplasmaNonUnit, 1.0, T, X)
    tp.execute(ctx)
    tr = getattr(tp, "transport", None)
    out["trsm"] = X.to_dense_local().cpu()
    out["trsm_xfers"] = tr.stats["xfers"] if tr is not None else 0
    # incremental-pivoting LU (tile DAG)
    L0 = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plrnt(ctx, L0, 3)
    Li = dp.incpiv_L_descriptor(ctx, L0, 8)
    IP = dp.incpiv_ipiv_descriptor(ctx, L0)
    tp = dp.getrf_incpiv_New(ctx, L0, Li, IP)
    info = tp.execute(ctx)
    tr = getattr(tp, "transport", None)
    out["incpiv"] = (info, L0.to_dense_local().cpu())
    out["incpiv_xfers"] = tr.stats["xfers"] if tr is not None else 0
    return out


def _loop_worker(rank, world):
    os.environ["DPLASMA_LOOPBACK"] = "1"
    import dplasma_amd as dp
    from dplasma_amd.parallel import comm
    assert comm.loopback()
    ctx = dp.init(device="cpu")
    assert ctx.loopback and ctx.urgent_group is not None
    return _algos(ctx, "cpu")


def _reference(dev):
    import dplasma_amd as dp
    ctx = dp.Context(device=dev)
    assert not ctx.loopback
    return _algos(ctx, dev)


def _compare(got, ref):
    assert {"DSEND", "XFER", "TRSM"} <= set(got["potrf_tasks"]), got["potrf_tasks"]
    assert "EXCH" in got["gemm_tasks"], got["gemm_tasks"]
    assert got["potrf"][0] == 0 == ref["potrf"][0]
    assert (got["potrf"][1] - ref["potrf"][1]).abs().max() < 1e-10
    assert (got["gemm"] - ref["gemm"]).abs().max() < 1e-10
    assert (got["trsm"] - ref["trsm"]).abs().max() < 1e-9
    assert got["trsm_xfers"] > 0, "the TRSM tile program moved nothing through the transport"
    assert got["incpiv"][0] == 0 == ref["incpiv"][0]
    assert (got["incpiv"][1] - ref["incpiv"][1]).abs().max() < 1e-10
    assert got["incpiv_xfers"] > 0, "the incpiv tile DAG moved nothing through the transport"


def test_loopback_cpu_gloo():
    out = run_distributed(_loop_worker, 1)
    _compare(out[0], _reference("cpu"))


_GPU_SCRIPT = r'''
import os, sys, json
sys.path.insert(0, os.environ["REPO"])
os.environ["DPLASMA_LOOPBACK"] = "1"
import torch, torch.distributed as dist
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
sys.path.insert(0, os.path.join(os.environ["REPO"], "tests"))
import test_loopback as T
import dplasma_amd as dp
from dplasma_amd.parallel import comm, p2p
calls = {"issue_gpu": 0, "start_p2p": 0}
_orig_issue = p2p.Transport._issue_gpu
def _issue(self, xs, stream):
    calls["issue_gpu"] += 1
    return _orig_issue(self, xs, stream)
p2p.Transport._issue_gpu = _issue
_orig_start = comm.start_p2p
def _start(*a, **k):
    calls["start_p2p"] += 1
    return _orig_start(*a, **k)
comm.start_p2p = _start
ctx = dp.init()
assert ctx.loopback and dist.get_backend() == "nccl"
got = T._algos(ctx, "cuda")
torch.save(got, os.environ["OUT"])
print(json.dumps(calls))
dist.destroy_process_group()
'''


@pytest.mark.gpu
def test_loopback_gpu_rccl(tmp_path):
    """World-1 NCCL group: every exchange is a real RCCL self send / receive."""
    import subprocess
    import sys
    from helpers import free_port
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "lb.py"
    script.write_text(_GPU_SCRIPT)
    env = dict(os.environ, REPO=repo, OUT=str(tmp_path / "out.pt"), MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
               HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    r = subprocess.run([sys.executable, str(script)], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    import json
    calls = json.loads(r.stdout.strip().splitlines()[-1])
    assert calls["issue_gpu"] > 0 and calls["start_p2p"] > 0, calls
    got = torch.load(str(tmp_path / "out.pt"), weights_only=True)
    _compare(got, _reference("cuda"))
