"""Tracing (Chrome trace of batched launches), DOT dumps of tile DAGs, dplasma_info options
(tests/testing_info.c), and the DPLASMA_TRACE_KERNELS launch log."""
import json
import os
import subprocess
import sys

import pytest
import torch

import dplasma_amd as dp
from dplasma_amd.models import qr_panel
from helpers import run_distributed


@pytest.fixture(scope="module")
def ctx():
    return dp.init(device="cpu")


def _qr(ctx, N=48, NB=16):
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plrnt(ctx, A, 1)
    T = dp.block_cyclic(ctx, torch.float64, 4, NB, A.mt * 4, N)
    dp.geqrf(ctx, A, T)


def test_trace_records_launches(ctx, tmp_path):
    tr = dp.profiling_start(ctx)
    _qr(ctx)                      # stacked-domain engine: panel / next / rest tasks
    with qr_panel.engine("tile"):
        _qr(ctx)                  # tile DAG: one launch per kernel kind and level
    tr.save_info("N", 48)
    dp.profiling_stop(ctx, str(tmp_path / "t.json"))
    d = json.load(open(tmp_path / "t.json"))
    names = {e["name"] for e in d["traceEvents"] if e.get("ph") == "X"}
    assert "geqrf" in names
    assert any("qr_panel" in n for n in names) and any("qr_rest" in n for n in names)
    assert any("geqrt" in n for n in names) and any("tsmqr" in n for n in names)
    assert d["otherData"]["N"] == 48
    s = tr.summary()
    assert s["geqrf"]["count"] >= 2 and s["geqrf"]["total_us"] > 0
    assert ctx.profiling is None


def test_dot_dump(ctx, tmp_path):
    p = str(tmp_path / "g.dot")
    dp.dot_start(ctx, p)
    with qr_panel.engine("tile"):   # DOT dumps are of tile DAGs
        _qr(ctx)
    dp.dot_stop(ctx)
    txt = open(p).read()
    assert txt.startswith('digraph "geqrf"') and "->" in txt and "geqrt" in txt


def test_info_api():
    inf = dp.info_create()
    assert dp.info_set(inf, "DPLASMA:GEMM:GPU:b", "4") == 0
    assert dp.info_set(inf, "k2", "v2") == 0
    assert dp.info_get(inf, "DPLASMA:GEMM:GPU:b") == "4"
    assert dp.info_get_nkeys(inf) == 2 and dp.info_get_nthkey(inf, 1) == "k2"
    assert dp.info_delete(inf, "k2") == 0 and dp.info_delete(inf, "k2") == -1
    assert dp.info_get(inf, "k2") is None
    dp.info_free(inf)
    assert dp.info_get_nkeys(inf) == 0


def test_trace_kernels_env():
    code = ("import torch, dplasma_amd as dp; c = dp.init(device='cpu'); "
            "A = dp.block_cyclic(c, torch.float64, 8, 8, 16, 16); dp.plrnt(c, A, 1)")
    env = dict(os.environ, DPLASMA_TRACE_KERNELS="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stderr
    assert "taskpool: plrnt" in r.stderr


def _worker(rank, world, path):
    ctx = dp.init(device="cpu", P=2)
    dp.profiling_start(ctx)
    _qr(ctx, 64, 16)
    dp.profiling_stop(ctx, path)
    return 0


def test_trace_distributed_gather(tmp_path):
    p = str(tmp_path / "d.json")
    run_distributed(_worker, 2, p)
    d = json.load(open(p))
    pids = {e["pid"] for e in d["traceEvents"]}
    assert pids == {0, 1}
    assert any(e.get("cat") == "comm" for e in d["traceEvents"])


@pytest.mark.gpu
def test_gpu_trace_streams(tmp_path):
    g = dp.init(device="cuda:0")
    tr = dp.profiling_start(g)
    A = dp.block_cyclic(g, torch.float64, 128, 128, 1024, 1024)
    dp.plrnt(g, A, 1)
    T = dp.block_cyclic(g, torch.float64, 32, 128, A.mt * 32, 1024)
    dp.geqrf(g, A, T)
    dp.profiling_stop(g, str(tmp_path / "g.json"))
    d = json.load(open(tmp_path / "g.json"))
    ev = [e for e in d["traceEvents"] if e.get("ph") == "X"]
    tracks = {e["tid"] for e in ev if e["cat"] in ("dag", "task")}
    assert {"panel", "update"} <= tracks
    assert all(e["dur"] >= 0 for e in ev)
