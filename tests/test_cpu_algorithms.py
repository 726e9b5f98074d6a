"""CPU reference path: algorithms on a single rank vs dense PyTorch fp64."""
import pytest
import torch

import dplasma_amd as dp
from helpers import DTYPES, rel_err, tol


@pytest.fixture(scope="module")
def ctx():
    return dp.init(device="cpu")


@pytest.mark.parametrize("prec", list("sdcz"))
@pytest.mark.parametrize("uplo", [dp.dplasmaLower, dp.dplasmaUpper])
def test_potrf(ctx, prec, uplo):
    dt = DTYPES[prec]
    N, NB = 378, 93
    A = dp.block_cyclic(ctx, dt, NB, NB, N, N)
    dp.plghe(ctx, float(N), uplo, A, 3872)
    A0 = A.like()
    dp.lacpy(ctx, dp.dplasmaUpperLower, A, A0)
    info = dp.potrf(ctx, uplo, A)
    assert info == 0
    ok, res = dp.check_potrf(ctx, uplo, A, A0)
    assert ok, res


def test_potrf_not_spd(ctx):
    N, NB = 64, 16
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plghe(ctx, 0.0, dp.dplasmaLower, A, 1)  # no bump -> indefinite
    info = dp.potrf(ctx, dp.dplasmaLower, A)
    assert info > 0


@pytest.mark.parametrize("prec", list("dz"))
@pytest.mark.parametrize("ta", [dp.dplasmaNoTrans, dp.dplasmaTrans, dp.dplasmaConjTrans])
@pytest.mark.parametrize("tb", [dp.dplasmaNoTrans, dp.dplasmaTrans, dp.dplasmaConjTrans])
def test_gemm(ctx, prec, ta, tb):
    dt = DTYPES[prec]
    M, N, K, NB = 106, 83, 97, 56
    am, an = (M, K) if ta == dp.dplasmaNoTrans else (K, M)
    bm, bn = (K, N) if tb == dp.dplasmaNoTrans else (N, K)
    A = dp.block_cyclic(ctx, dt, NB, NB, am, an)
    B = dp.block_cyclic(ctx, dt, NB, NB, bm, bn)
    C = dp.block_cyclic(ctx, dt, NB, NB, M, N)
    dp.plrnt(ctx, A, 3872)
    dp.plrnt(ctx, B, 4674)
    dp.plrnt(ctx, C, 2873)
    a, b, c = A.to_dense_local(), B.to_dense_local(), C.to_dense_local()
    op = {dp.dplasmaNoTrans: lambda x: x, dp.dplasmaTrans: lambda x: x.T, dp.dplasmaConjTrans: lambda x: x.conj().T}
    ref = 0.51 * op[ta](a) @ op[tb](b) - 0.42 * c
    dp.gemm(ctx, ta, tb, 0.51, A, B, -0.42, C)
    assert rel_err(C.to_dense_local(), ref) < tol(dt)


@pytest.mark.parametrize("norm", [dp.dplasmaMaxNorm, dp.dplasmaOneNorm, dp.dplasmaInfNorm, dp.dplasmaFrobeniusNorm])
def test_norms(ctx, norm):
    M, N, NB = 87, 61, 16
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, M, N)
    dp.plrnt(ctx, A, 5)
    a = A.to_dense_local()
    ref = {dp.dplasmaMaxNorm: a.abs().max(), dp.dplasmaOneNorm: a.abs().sum(0).max(),
           dp.dplasmaInfNorm: a.abs().sum(1).max(), dp.dplasmaFrobeniusNorm: a.norm()}[norm].item()
    assert abs(dp.lange(ctx, norm, A) - ref) <= 1e-12 * ref


@pytest.mark.parametrize("uplo", [dp.dplasmaLower, dp.dplasmaUpper])
@pytest.mark.parametrize("norm", [dp.dplasmaMaxNorm, dp.dplasmaOneNorm, dp.dplasmaInfNorm, dp.dplasmaFrobeniusNorm])
def test_lanhe(ctx, uplo, norm):
    N, NB = 70, 16
    A = dp.block_cyclic(ctx, torch.complex128, NB, NB, N, N)
    dp.plghe(ctx, 3.0, dp.dplasmaUpperLower, A, 5)
    a = A.to_dense_local()
    ref = {dp.dplasmaMaxNorm: a.abs().max(), dp.dplasmaOneNorm: a.abs().sum(0).max(),
           dp.dplasmaInfNorm: a.abs().sum(1).max(), dp.dplasmaFrobeniusNorm: a.norm()}[norm].item()
    # wipe the other triangle: lanhe must not read it
    other = dp.dplasmaUpper if uplo == dp.dplasmaLower else dp.dplasmaLower
    from dplasma_amd.ops import tile_ops as ops
    from dplasma_amd.models.aux import local_tile_batch
    ops.laset(4 if uplo == dp.dplasmaLower else 3, 7.0, 7.0, A.data, A.ld, local_tile_batch(A))
    got = dp.lanhe(ctx, norm, uplo, A)
    assert abs(got - ref) <= 1e-12 * ref


def test_lantr(ctx):
    N, NB = 45, 10
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plrnt(ctx, A, 11)
    a = A.to_dense_local()
    t = a.tril()
    t.fill_diagonal_(1.0)
    assert abs(dp.lantr(ctx, dp.dplasmaOneNorm, dp.dplasmaLower, dp.dplasmaUnit, A) - t.abs().sum(0).max().item()) < 1e-12


@pytest.mark.parametrize("prec", list("dz"))
@pytest.mark.parametrize("uplo", [dp.dplasmaLower, dp.dplasmaUpper])
def test_potrf_blocked_tile_kernel(ctx, prec, uplo, monkeypatch):
    """Diagonal tiles factored as 128-wide right-looking steps (POTRF + TRSM + masked GEMM)."""
    monkeypatch.setenv("DPLASMA_POTRF_TILE", "blocked")
    dt = DTYPES[prec]
    N, NB = 700, 300   # tiles of 300 -> steps 128, 128, 44; ragged 100 last tile
    A = dp.block_cyclic(ctx, dt, NB, NB, N, N)
    dp.plghe(ctx, float(N), uplo, A, 3872)
    A0 = A.like()
    dp.lacpy(ctx, dp.dplasmaUpperLower, A, A0)
    assert dp.potrf(ctx, uplo, A) == 0
    ok, res = dp.check_potrf(ctx, uplo, A, A0)
    assert ok, res
