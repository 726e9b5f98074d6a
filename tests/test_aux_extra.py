"""Generators (pltmg / latms / plrnt diagdom), lanm2, print, apply / map2."""
import io

import pytest
import torch

import dplasma_amd as dp
from dplasma_amd.models import generators as G
from helpers import rel_err, run_distributed


@pytest.fixture(scope="module")
def ctx():
    return dp.init(device="cpu")


@pytest.mark.parametrize("dt", [torch.float64, torch.complex128])
def test_pltmg_all_types_tiling_independent(ctx, dt):
    N = 24
    for t in range(43):
        A = dp.block_cyclic(ctx, dt, 7, 7, N, N)
        B = dp.block_cyclic(ctx, dt, 5, 5, N, N)
        r1, r2 = dp.pltmg(ctx, t, A, 11), dp.pltmg(ctx, t, B, 11)
        assert r1 == r2
        if t in G.UNAVAILABLE or t == dp.dplasmaMatrixHadamard:  # Hadamard needs a power-of-two order
            assert r1 == -2
            continue
        assert r1 == 0, t
        assert torch.allclose(A.to_dense_local(), B.to_dense_local()), t


def test_pltmg_properties(ctx):
    A = dp.block_cyclic(ctx, torch.float64, 8, 8, 16, 16)
    dp.pltmg(ctx, dp.dplasmaMatrixHilb, A, 1)
    a = A.to_dense_local()
    assert abs(a[2, 3] - 1 / 6) < 1e-15
    for t, gram in ((dp.dplasmaMatrixOrthog, 1.0), (dp.dplasmaMatrixHadamard, 16.0), (dp.dplasmaMatrixHouse, 1.0)):
        dp.pltmg(ctx, t, A, 3)
        a = A.to_dense_local()
        assert (a @ a.T - gram * torch.eye(16, dtype=torch.float64)).abs().max() < 1e-12
    dp.pltmg(ctx, dp.dplasmaMatrixToeppd, A, 3)
    a = A.to_dense_local()
    assert torch.allclose(a, a.T) and torch.linalg.eigvalsh(a).min() > -1e-10


def test_latms_condition(ctx):
    A = dp.block_cyclic(ctx, torch.float64, 8, 8, 32, 32)
    dp.latms(ctx, dp.dplasmaGeneral, 1e4, A, 5)
    s = torch.linalg.svdvals(A.to_dense_local())
    assert abs(s[0] / s[-1] - 1e4) < 1e-6 * 1e4 and abs(s[0] - 1) < 1e-12


def test_plrnt_diagdom(ctx):
    A = dp.block_cyclic(ctx, torch.float64, 8, 8, 20, 20)
    B = dp.block_cyclic(ctx, torch.float64, 8, 8, 20, 20)
    dp.plrnt(ctx, 1, A, 7)
    dp.plrnt(ctx, B, 7)
    d = A.to_dense_local() - B.to_dense_local()
    assert torch.allclose(d, 20.0 * torch.eye(20, dtype=torch.float64))


def test_lanm2(ctx):
    A = dp.block_cyclic(ctx, torch.float64, 8, 8, 30, 20)
    dp.plrnt(ctx, A, 3)
    info = []
    est = dp.lanm2(ctx, A, info)
    assert info[0] > 0
    assert abs(est - float(torch.linalg.matrix_norm(A.to_dense_local(), 2))) < 1e-6 * est


def test_print_apply_map2(ctx):
    A = dp.block_cyclic(ctx, torch.float64, 4, 4, 6, 6)
    dp.plrnt(ctx, A, 1)
    buf = io.StringIO()
    dp.print(ctx, dp.dplasmaUpperLower, A, file=buf)
    assert "A(1,1)" in buf.getvalue()
    B = dp.block_cyclic(ctx, torch.float64, 4, 4, 6, 6)
    dp.apply(ctx, dp.dplasmaUpperLower, B, lambda t, uplo, m, n, args: t.fill_(args), 2.0)
    assert (B.to_dense_local() == 2.0).all()
    dp.map2(ctx, dp.dplasmaUpperLower, dp.dplasmaTrans, A, B, lambda a, b, uplo, m, n, args: b.add_(a), None)
    assert rel_err(B.to_dense_local(), 2.0 + A.to_dense_local().T) < 1e-15


def _gen_worker(rank, world):
    import dplasma_amd as dp
    ctx = dp.init(device="cpu", P=2)
    A = dp.block_cyclic(ctx, torch.float64, 5, 5, 17, 17)
    dp.pltmg(ctx, dp.dplasmaMatrixFiedler, A, 4)
    return A.to_dense_local(), dp.lanm2(ctx, A)


def test_generators_distributed(ctx):
    out = run_distributed(_gen_worker, 4)
    A = dp.block_cyclic(ctx, torch.float64, 5, 5, 17, 17)
    dp.pltmg(ctx, dp.dplasmaMatrixFiedler, A, 4)
    assert rel_err(sum(out[r][0] for r in range(4)), A.to_dense_local()) < 1e-15
    assert abs(out[0][1] - float(torch.linalg.matrix_norm(A.to_dense_local(), 2))) < 1e-6 * out[0][1]


@pytest.mark.gpu
def test_pltmg_gpu_matches_cpu():
    """pltmg evaluated on the GPU (device formulas, GPU LCG base) equals the CPU evaluation."""
    cg, cc = dp.init(device="cuda:0"), dp.init(device="cpu")
    for t in range(43):
        A = dp.block_cyclic(cg, torch.float64, 16, 16, 72, 72)
        B = dp.block_cyclic(cc, torch.float64, 16, 16, 72, 72)
        r1, r2 = dp.pltmg(cg, t, A, 5), dp.pltmg(cc, t, B, 5)
        assert r1 == r2
        if r1 == 0:
            b = B.to_dense_local()
            # relative: Demmel spans 1 .. 1e14 (GPU and CPU pow differ in the last bit)
            assert (A.to_dense_local().cpu() - b).abs().max() <= 1e-12 * max(1.0, float(b.abs().max())), t
