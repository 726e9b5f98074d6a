"""Memory-capped Cholesky (models/potrf_ooc.py): a bounded tile arena with LRU eviction and
write-back, the analogue of the reference's low-memory test (tests/Testings.cmake:147, 21 device
blocks).  CPU: the arena logic on a CPU context; GPU: a host-resident matrix on a GPU context."""
import pytest
import torch

import dplasma_amd as dp
from dplasma_amd.models.potrf_ooc import potrf_ooc_New


def _run(ctx, N, NB, uplo, nblocks, host=True):
    A = dp.TiledMatrix(torch.float64, NB, NB, N, N, device="cpu")
    cctx = dp.Context(device="cpu")
    dp.plghe(cctx, float(N), uplo, A, 3872)
    A0 = A.like()
    A0.data.copy_(A.data)
    tp = potrf_ooc_New(ctx, uplo, A, nblocks)
    info = tp.execute(ctx)
    ok, res = dp.check_potrf(cctx, uplo, A, A0)
    return info, ok, res, tp.cache


@pytest.mark.parametrize("nblocks", [3, 5, 21])
@pytest.mark.parametrize("uplo", [dp.dplasmaLower, dp.dplasmaUpper])
def test_potrf_capped_cpu(nblocks, uplo):
    ctx = dp.Context(device="cpu")
    info, ok, res, cache = _run(ctx, 320, 32, uplo, nblocks)
    assert info == 0 and ok, res
    assert cache.evictions > 0 and cache.writebacks > 0   # 55 tiles through <= 21 slots


def test_potrf_capped_info_cpu():
    ctx = dp.Context(device="cpu")
    N, NB = 96, 32
    A = dp.TiledMatrix(torch.float64, NB, NB, N, N, device="cpu")
    A.from_dense(torch.eye(N, dtype=torch.float64))
    A.tile(1, 1)[5, 5] = -1.0
    assert potrf_ooc_New(ctx, dp.dplasmaLower, A, 3).execute(ctx) == 32 + 6


@pytest.mark.gpu
def test_potrf_lowmem_gpu():
    """Host matrix, GPU context, 21 device blocks (the reference's 1gpu_lowmem configuration, scaled)."""
    ctx = dp.Context(device="cuda:0")
    info, ok, res, cache = _run(ctx, 1600, 160, dp.dplasmaLower, 21)
    assert info == 0 and ok, res
    assert cache.evictions > 0
    # the generic entry point dispatches a host matrix on a GPU context to the capped variant
    A = dp.TiledMatrix(torch.float64, 160, 160, 800, 800, device="cpu")
    dp.plghe(dp.Context(device="cpu"), 800.0, dp.dplasmaLower, A, 7)
    assert dp.potrf(ctx, dp.dplasmaLower, A) == 0


@pytest.mark.parametrize("uplo", [dp.dplasmaLower, dp.dplasmaUpper])
@pytest.mark.parametrize("hnb", [16, 24])
def test_potrf_recursive_cpu(hnb, uplo):
    """setrecursive(hnb): every diagonal-tile factorisation, panel solve and trailing update of a tile
    larger than hnb runs as a sub-taskpool of hnb tiles (POTRF / TRSM / HERK / GEMM incarnations)."""
    ctx = dp.Context(device="cpu")
    N, NB = 200, 64
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plghe(ctx, float(N), uplo, A, 3872)
    A0 = A.like()
    dp.lacpy(ctx, dp.dplasmaUpperLower, A, A0)
    tp = dp.dpotrf_New(ctx, uplo, A)
    dp.dpotrf_setrecursive(tp, hnb)
    assert tp.execute(ctx) == 0
    ok, res = dp.check_potrf(ctx, uplo, A, A0)
    assert ok, res
    subs = tp._rec_subs
    pot = [k for k in subs if not isinstance(k[0], str)]
    assert len(pot) == sum(A.tile_rows(k) > hnb for k in range(A.nt))  # one per large diagonal tile
    assert any(k[0] == "trsm" for k in subs) and any(k[0] == "upd" for k in subs)
    sub = subs[pot[0]][0]
    assert any(t.name.startswith("POTRF(1)") for t in sub.tasks)   # the tile really was re-tiled
    names = {type(v[0]).__name__ for v in subs.values()}
    assert names == {"Taskpool"}


def test_potrf_recursive_info_cpu():
    ctx = dp.Context(device="cpu")
    N, NB = 96, 48
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    A.from_dense(torch.eye(N, dtype=torch.float64))
    A.tile(1, 1)[20, 20] = -1.0
    tp = dp.dpotrf_New(ctx, dp.dplasmaLower, A)
    dp.dpotrf_setrecursive(tp, 16)
    assert tp.execute(ctx) == 48 + 21


@pytest.mark.gpu
@pytest.mark.parametrize("uplo", [dp.dplasmaLower, dp.dplasmaUpper])
def test_potrf_recursive_gpu(uplo):
    ctx = dp.Context(device="cuda:0")
    N, NB = 2048, 512
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plghe(ctx, float(N), uplo, A, 3872)
    A0 = A.like()
    dp.lacpy(ctx, dp.dplasmaUpperLower, A, A0)
    tp = dp.dpotrf_New(ctx, uplo, A)
    dp.dpotrf_setrecursive(tp, 128)
    assert tp.execute(ctx) == 0
    ok, res = dp.check_potrf(ctx, uplo, A, A0)
    assert ok, res
    assert any(k[0] == "trsm" for k in tp._rec_subs) and any(k[0] == "upd" for k in tp._rec_subs)
