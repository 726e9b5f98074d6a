"""DTD insert-task front end: generic bodies, hazards, distribution, and the DTD Cholesky."""
import pytest
import torch

import dplasma_amd as dp
from dplasma_amd.models.dtd_potrf import potrf_dtd
from dplasma_amd.runtime import dtd
from helpers import rel_err, run_distributed


@pytest.fixture(scope="module")
def ctx():
    return dp.init(device="cpu")


def test_dtd_program_order_semantics(ctx):
    """A chain of read/write tasks on shared tiles must observe program order (RAW/WAR/WAW)."""
    A = dp.block_cyclic(ctx, torch.float64, 4, 4, 8, 8)
    tp = dtd.taskpool_new(ctx)
    T = dtd.tile_of

    def setv(a, v):
        a.fill_(v)

    def axpy(x, y, alpha):  # y += alpha * x
        y.add_(alpha * x)
    tp.insert_task(setv, (T(A, 0, 0), dtd.OUTPUT), 1.0)
    tp.insert_task(setv, (T(A, 1, 1), dtd.OUTPUT), 2.0)
    tp.insert_task(axpy, (T(A, 0, 0), dtd.INPUT), (T(A, 1, 1), dtd.INOUT), 3.0)   # A11 = 2 + 3 = 5
    tp.insert_task(setv, (T(A, 0, 0), dtd.OUTPUT), 7.0)                            # WAR on A00
    tp.insert_task(axpy, (T(A, 1, 1), dtd.INPUT), (T(A, 0, 0), dtd.INOUT), 1.0)   # A00 = 7 + 5 = 12
    tp.execute()
    a = A.to_dense_local()
    assert (a[:4, :4] == 12).all() and (a[4:, 4:] == 5).all()


@pytest.mark.parametrize("uplo", [dp.dplasmaLower, dp.dplasmaUpper])
@pytest.mark.parametrize("dt", [torch.float64, torch.complex128])
def test_potrf_dtd(ctx, uplo, dt):
    N, NB = 70, 16
    A = dp.block_cyclic(ctx, dt, NB, NB, N, N)
    dp.plghe(ctx, float(N), dp.dplasmaUpperLower, A, 3)
    a = A.to_dense_local()
    assert potrf_dtd(ctx, uplo, A) == 0
    L = torch.linalg.cholesky(a)
    got = A.to_dense_local()
    if uplo == dp.dplasmaLower:
        assert rel_err(torch.tril(got), L) < 1e-12
    else:
        assert rel_err(torch.triu(got), L.conj().T) < 1e-12


def _worker(rank, world, P):
    import dplasma_amd as dp
    from dplasma_amd.models.dtd_potrf import potrf_dtd
    ctx = dp.init(device="cpu", P=P)
    A = dp.block_cyclic(ctx, torch.float64, 16, 16, 70, 70)
    dp.plghe(ctx, 70.0, dp.dplasmaUpperLower, A, 3)
    return potrf_dtd(ctx, dp.dplasmaLower, A), A.to_dense_local()


@pytest.mark.parametrize("world,P", [(2, 1), (4, 2)])
def test_potrf_dtd_distributed(world, P):
    out = run_distributed(_worker, world, P)
    ctx = dp.init(device="cpu")
    A = dp.block_cyclic(ctx, torch.float64, 16, 16, 70, 70)
    dp.plghe(ctx, 70.0, dp.dplasmaUpperLower, A, 3)
    L = torch.linalg.cholesky(A.to_dense_local())
    assert all(out[r][0] == 0 for r in range(world))
    assert rel_err(torch.tril(sum(out[r][1] for r in range(world))), L) < 1e-12


@pytest.mark.gpu
def test_gpu_potrf_dtd():
    g = dp.init(device="cuda:0")
    N, NB = 1000, 128
    A = dp.block_cyclic(g, torch.float64, NB, NB, N, N)
    dp.plghe(g, float(N), dp.dplasmaUpperLower, A, 3)
    a = A.to_dense_local().cpu()
    assert potrf_dtd(g, dp.dplasmaLower, A) == 0
    assert rel_err(torch.tril(A.to_dense_local().cpu()), torch.linalg.cholesky(a)) < 1e-11
