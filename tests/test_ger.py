"""Rank-1 updates gerc / geru (src/zger.jdf) and the setrecursive hints."""
import pytest
import torch

import dplasma_amd as dp
from helpers import DTYPES, run_distributed


@pytest.fixture(scope="module")
def ctx():
    return dp.init(device="cpu")


def _vecs(ctx, dt, M, N, NB):
    A = dp.block_cyclic(ctx, dt, NB, NB, M, N)
    X = dp.block_cyclic(ctx, dt, NB, NB, M, 1)
    Y = dp.block_cyclic(ctx, dt, NB, NB, N, 1)
    for s, T in enumerate((A, X, Y)):
        dp.plrnt(ctx, T, 10 + s)
    return A, X, Y


@pytest.mark.parametrize("prec", list("sdcz"))
def test_gerc_geru(ctx, prec):
    dt = DTYPES[prec]
    A, X, Y = _vecs(ctx, dt, 45, 37, 16)
    a, x, y = (T.to_dense_local() for T in (A, X, Y))
    dp.gerc(ctx, 0.5, X, Y, A)
    ref = a + 0.5 * x @ y.conj().T
    tol = 1e-5 if prec in "sc" else 1e-13
    assert (A.to_dense_local() - ref).abs().max() < tol
    dp.geru(ctx, -1.0, X, Y, A)
    assert (A.to_dense_local() - (ref - x @ y.T)).abs().max() < tol


def _worker(rank, world, P):
    c = dp.init(device="cpu", P=P)
    A, X, Y = _vecs(c, torch.float64, 50, 40, 16)
    dp.ger(c, 2.0, X, Y, A)
    return A.to_dense_local(), X.to_dense_local(), Y.to_dense_local()


def test_ger_distributed(ctx):
    out = run_distributed(_worker, 4, 2)
    a = sum(o[0] for o in out.values())
    A, X, Y = _vecs(ctx, torch.float64, 50, 40, 16)
    ref = A.to_dense_local() + 2.0 * X.to_dense_local() @ Y.to_dense_local().T
    assert (a - ref).abs().max() < 1e-13


def test_setrecursive_hint(ctx):
    A = dp.block_cyclic(ctx, torch.float64, 16, 16, 32, 32)
    dp.plghe(ctx, 32.0, dp.dplasmaUpperLower, A, 1)
    tp = dp.dpotrf_New(ctx, dp.dplasmaLower, A)
    assert dp.dpotrf_setrecursive(tp, 8) == 0 and tp.recursive_nb == 8
    tp.execute(ctx)
