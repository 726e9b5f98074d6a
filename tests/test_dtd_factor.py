"""DTD tile QR (geqrf_dtd, untied) and incremental-pivoting LU (getrf_incpiv_dtd): the same tile kernels as
the PTG-style tile engines, so the results must match them (tests/testing_zgeqrf_dtd*.c,
testing_zgetrf_incpiv_dtd.c)."""
import pytest
import torch

import dplasma_amd as dp
from dplasma_amd.models import qr_panel
from helpers import rel_err, run_distributed


@pytest.fixture(scope="module")
def ctx():
    return dp.init(device="cpu")


def _qr_pair(ctx, dt, M, N, NB, IB, seed=5):
    A = dp.block_cyclic(ctx, dt, NB, NB, M, N)
    dp.plrnt(ctx, A, seed)
    T = dp.block_cyclic(ctx, dt, IB, NB, A.mt * IB, A.nt * NB, name="T")
    return A, T


def _normal_eq_residual(a0, r):
    """||A^H A - R^H R|| / (||A||^2 N eps): a QR check that needs no Q (any V/T storage)."""
    K = min(a0.shape)
    R = torch.triu(r[:K])
    eps = torch.finfo(a0.real.dtype if a0.is_complex() else a0.dtype).eps
    g = a0.conj().T @ a0
    return float((g - R.conj().T @ R).abs().max() / (a0.abs().max() ** 2 * max(a0.shape) * eps))


@pytest.mark.parametrize("dt", [torch.float64, torch.complex128])
@pytest.mark.parametrize("untied", [False, True])
def test_geqrf_dtd_matches_tile_engine(ctx, dt, untied):
    M, N, NB, IB = 150, 118, 32, 8
    A, T = _qr_pair(ctx, dt, M, N, NB, IB)
    B, TB = _qr_pair(ctx, dt, M, N, NB, IB)
    a0 = A.to_dense_local().clone()
    (dp.geqrf_dtd_untied if untied else dp.geqrf_dtd)(ctx, A, T, window=17)
    with qr_panel.engine("tile"):
        dp.geqrf(ctx, B, TB)
    assert rel_err(A.to_dense_local(), B.to_dense_local()) < 1e-12
    assert rel_err(T.to_dense_local(), TB.to_dense_local()) < 1e-12
    assert _normal_eq_residual(a0, A.to_dense_local()) < 60
    # the factors feed the reference-layout apply: Q from ungqr is orthonormal and Q R = A
    Q = dp.block_cyclic(ctx, dt, NB, NB, M, min(M, N), name="Q")
    dp.ungqr(ctx, A, T, Q)
    q = Q.to_dense_local()
    assert rel_err(q @ torch.triu(A.to_dense_local()[:min(M, N)]), a0) < 1e-12


def test_geqrf_dtd_New_taskpool(ctx):
    A, T = _qr_pair(ctx, torch.float64, 96, 96, 32, 8)
    B, TB = _qr_pair(ctx, torch.float64, 96, 96, 32, 8)
    tp = dp.geqrf_dtd_New(ctx, A, T)
    ctx.add_taskpool(tp)
    ctx.start()
    ctx.wait()
    with qr_panel.engine("tile"):
        dp.geqrf(ctx, B, TB)
    assert rel_err(A.to_dense_local(), B.to_dense_local()) < 1e-12


@pytest.mark.parametrize("dt", [torch.float64, torch.complex64])
def test_getrf_incpiv_dtd_matches_tile_engine(ctx, dt):
    N, NB, IB = 140, 32, 8
    out = []
    for dtd_path in (True, False):
        A = dp.block_cyclic(ctx, dt, NB, NB, N, N)
        dp.plrnt(ctx, A, 7)
        L = dp.incpiv_L_descriptor(ctx, A, IB)
        IP = dp.incpiv_ipiv_descriptor(ctx, A)
        info = (dp.getrf_incpiv_dtd if dtd_path else dp.getrf_incpiv)(ctx, A, L, IP)
        assert info == 0
        out.append((A.to_dense_local(), L.to_dense_local(), IP.to_dense_local()))
    tol = 1e-12 if dt == torch.float64 else 1e-5
    assert rel_err(out[0][0], out[1][0]) < tol
    assert rel_err(out[0][1], out[1][1]) < tol
    assert torch.equal(out[0][2], out[1][2])


def _worker_qr(rank, world, P):
    import dplasma_amd as dp
    ctx = dp.init(device="cpu", P=P)
    A = dp.block_cyclic(ctx, torch.float64, 24, 24, 100, 72)
    dp.plrnt(ctx, A, 5)
    T = dp.block_cyclic(ctx, torch.float64, 8, 24, A.mt * 8, A.nt * 24, name="T")
    dp.geqrf_dtd(ctx, A, T, window=13)
    return A.to_dense_local()


@pytest.mark.parametrize("world,P", [(2, 2), (4, 2)])
def test_geqrf_dtd_distributed(world, P):
    out = run_distributed(_worker_qr, world, P)
    ctx = dp.init(device="cpu")
    A = dp.block_cyclic(ctx, torch.float64, 24, 24, 100, 72)
    dp.plrnt(ctx, A, 5)
    T = dp.block_cyclic(ctx, torch.float64, 8, 24, A.mt * 8, A.nt * 24, name="T")
    with qr_panel.engine("tile"):
        dp.geqrf(ctx, A, T)
    got = sum(out[r] for r in range(world))
    assert rel_err(got, A.to_dense_local()) < 1e-12


@pytest.mark.gpu
def test_gpu_geqrf_and_getrf_incpiv_dtd():
    g = dp.init(device="cuda:0")
    M, N, NB, IB = 700, 520, 128, 32
    A, T = _qr_pair(g, torch.float64, M, N, NB, IB)
    a0 = A.to_dense_local().cpu()
    dp.geqrf_dtd(g, A, T)
    assert _normal_eq_residual(a0, A.to_dense_local().cpu()) < 60
    # T carries the per-tile layout tag: ungqr must take the tile apply, not the stacked-domain engine
    Q = dp.block_cyclic(g, torch.float64, NB, NB, M, N, name="Q")
    dp.ungqr(g, A, T, Q)
    q, r = Q.to_dense_local().cpu(), A.to_dense_local().cpu()
    assert rel_err(q @ torch.triu(r[:N]), a0) < 1e-12
    out = []
    for dtd_path in (True, False):
        B = dp.block_cyclic(g, torch.float64, NB, NB, 600, 600)
        dp.plrnt(g, B, 9)
        L = dp.incpiv_L_descriptor(g, B, IB)
        IP = dp.incpiv_ipiv_descriptor(g, B)
        assert (dp.getrf_incpiv_dtd if dtd_path else dp.getrf_incpiv)(g, B, L, IP) == 0
        out.append((B.to_dense_local().cpu(), IP.to_dense_local().cpu()))
    assert rel_err(out[0][0], out[1][0]) < 1e-12
    assert torch.equal(out[0][1], out[1][1])
