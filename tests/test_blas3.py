"""BLAS3 + Cholesky drivers vs dense PyTorch references (CPU path; same code runs on GPU)."""
import pytest
import torch

import dplasma_amd as dp
from helpers import DTYPES, rel_err, tol

OP = {111: lambda x: x, 112: lambda x: x.T, 113: lambda x: x.conj().T}


@pytest.fixture(scope="module")
def ctx():
    return dp.init(device="cpu")


def _mat(ctx, dt, m, n, nb, seed, kind="rnt", bump=0.0):
    A = dp.block_cyclic(ctx, dt, nb, nb, m, n)
    if kind == "rnt":
        dp.plrnt(ctx, A, seed)
    else:
        dp.plghe(ctx, bump, dp.dplasmaUpperLower, A, seed)
    return A


def _tri(a, uplo, diag):
    t = a.tril() if uplo == dp.dplasmaLower else a.triu()
    if diag == dp.dplasmaUnit:
        t = t - torch.diag_embed(torch.diagonal(t)) + torch.eye(t.shape[0], dtype=t.dtype)
    return t


@pytest.mark.parametrize("prec", ["d", "z"])
@pytest.mark.parametrize("side", [141, 142])
@pytest.mark.parametrize("uplo", [121, 122])
@pytest.mark.parametrize("trans", [111, 112, 113])
@pytest.mark.parametrize("diag", [131, 132])
def test_trsm_trmm(ctx, prec, side, uplo, trans, diag):
    dt = DTYPES[prec]
    M, N, NB = 60, 45, 16
    k = M if side == 141 else N
    A = _mat(ctx, dt, k, k, NB, 3, "ghe", bump=float(k))
    B = _mat(ctx, dt, M, N, NB, 4)
    a, b = A.to_dense_local(), B.to_dense_local()
    t = OP[trans](_tri(a, uplo, diag))
    ref = torch.linalg.solve(t, 0.7 * b) if side == 141 else torch.linalg.solve(t.T, (0.7 * b).T).T
    dp.trsm(ctx, side, uplo, trans, diag, 0.7, A, B)
    assert rel_err(B.to_dense_local(), ref) < 1e-12
    B2 = _mat(ctx, dt, M, N, NB, 4)
    dp.trmm(ctx, side, uplo, trans, diag, 0.7, A, B2)
    ref2 = 0.7 * t @ b if side == 141 else 0.7 * b @ t
    assert rel_err(B2.to_dense_local(), ref2) < 1e-12


@pytest.mark.parametrize("prec", ["d", "z"])
@pytest.mark.parametrize("side", [141, 142])
@pytest.mark.parametrize("uplo", [121, 122])
@pytest.mark.parametrize("herm", [False, True])
def test_symm_hemm(ctx, prec, side, uplo, herm):
    dt = DTYPES[prec]
    M, N, NB = 50, 37, 16
    k = M if side == 141 else N
    A = _mat(ctx, dt, k, k, NB, 5, "ghe", bump=1.0) if herm else _mat(ctx, dt, k, k, NB, 5)
    a = A.to_dense_local()
    tri = a.tril() if uplo == 122 else a.triu()
    if herm:
        full = tri + tri.conj().T - torch.diag_embed(torch.diagonal(tri))
    else:
        full = tri + tri.T - torch.diag_embed(torch.diagonal(tri))
    B = _mat(ctx, dt, M, N, NB, 6)
    C = _mat(ctx, dt, M, N, NB, 7)
    b, c = B.to_dense_local(), C.to_dense_local()
    (dp.hemm if herm else dp.symm)(ctx, side, uplo, 0.5, A, B, -0.3, C)
    ref = 0.5 * (full @ b if side == 141 else b @ full) - 0.3 * c
    assert rel_err(C.to_dense_local(), ref) < 1e-12


@pytest.mark.parametrize("uplo", [121, 122])
@pytest.mark.parametrize("trans", [111, 113])
@pytest.mark.parametrize("two", [False, True])
def test_herk_her2k(ctx, uplo, trans, two):
    dt = torch.complex128
    N, K, NB = 40, 30, 16
    am, an = (N, K) if trans == 111 else (K, N)
    A = _mat(ctx, dt, am, an, NB, 8)
    B = _mat(ctx, dt, am, an, NB, 9)
    C = _mat(ctx, dt, N, N, NB, 10, "ghe", bump=1.0)
    a, b, c = A.to_dense_local(), B.to_dense_local(), C.to_dense_local()
    opa = OP[trans]
    if two:
        alpha = 0.5 + 0.25j
        dp.her2k(ctx, uplo, trans, alpha, A, B, 0.7, C)
        if trans == 111:
            ref = alpha * a @ b.conj().T + alpha.conjugate() * b @ a.conj().T + 0.7 * c
        else:
            ref = alpha * a.conj().T @ b + alpha.conjugate() * b.conj().T @ a + 0.7 * c
    else:
        dp.herk(ctx, uplo, trans, 0.5, A, 0.7, C)
        ref = 0.5 * (a @ a.conj().T if trans == 111 else a.conj().T @ a) + 0.7 * c
    got = C.to_dense_local()
    sel = (lambda x: x.tril()) if uplo == 122 else (lambda x: x.triu())
    assert rel_err(sel(got), sel(ref)) < 1e-12


def test_syrk_syr2k(ctx):
    dt = torch.float64
    A = _mat(ctx, dt, 33, 21, 8, 1)
    B = _mat(ctx, dt, 33, 21, 8, 2)
    C = _mat(ctx, dt, 33, 33, 8, 3)
    a, b, c = A.to_dense_local(), B.to_dense_local(), C.to_dense_local()
    dp.syr2k(ctx, 122, 111, 0.3, A, B, 1.5, C)
    ref = 0.3 * (a @ b.T + b @ a.T) + 1.5 * c
    assert rel_err(C.to_dense_local().tril(), ref.tril()) < 1e-12
    C2 = _mat(ctx, dt, 21, 21, 8, 3)
    c2 = C2.to_dense_local()
    dp.syrk(ctx, 121, 112, 2.0, A, 0.0, C2)
    assert rel_err(C2.to_dense_local().triu(), (2.0 * a.T @ a).triu()) < 1e-12


def test_gerc(ctx):
    dt = torch.complex128
    X = _mat(ctx, dt, 37, 1, 8, 1)
    Y = _mat(ctx, dt, 29, 1, 8, 2)
    A = _mat(ctx, dt, 37, 29, 8, 3)
    x, y, a = X.to_dense_local(), Y.to_dense_local(), A.to_dense_local()
    dp.gerc(ctx, 0.5j, X, Y, A)
    assert rel_err(A.to_dense_local(), a + 0.5j * x @ y.conj().T) < 1e-12


@pytest.mark.parametrize("prec", ["d", "z"])
@pytest.mark.parametrize("uplo", [121, 122])
def test_cholesky_drivers(ctx, prec, uplo):
    dt = DTYPES[prec]
    N, NB, NRHS = 70, 16, 23
    A = _mat(ctx, dt, N, N, NB, 11, "ghe", bump=float(N))
    a = A.to_dense_local()
    B = _mat(ctx, dt, N, NRHS, NB, 12)
    b = B.to_dense_local()
    assert dp.posv(ctx, uplo, A, B) == 0
    assert rel_err(B.to_dense_local(), torch.linalg.solve(a, b)) < 1e-11
    A2 = _mat(ctx, dt, N, N, NB, 11, "ghe", bump=float(N))
    assert dp.poinv(ctx, uplo, A2) == 0
    inv = torch.linalg.inv(a)
    sel = (lambda x: x.tril()) if uplo == 122 else (lambda x: x.triu())
    assert rel_err(sel(A2.to_dense_local()), sel(inv)) < 1e-11


@pytest.mark.parametrize("uplo", [121, 122])
@pytest.mark.parametrize("diag", [131, 132])
def test_trtri_lauum(ctx, uplo, diag):
    dt = torch.float64
    N, NB = 53, 12
    A = _mat(ctx, dt, N, N, NB, 13, "ghe", bump=float(N))
    a = A.to_dense_local()
    dp.trtri(ctx, uplo, diag, A)
    t = _tri(a, uplo, diag)
    inv = torch.linalg.inv(t)
    got = A.to_dense_local()
    sel = (lambda x: x.tril(-1 if diag == 132 else 0)) if uplo == 122 else (lambda x: x.triu(1 if diag == 132 else 0))
    assert rel_err(sel(got), sel(inv)) < 1e-12
    A3 = _mat(ctx, dt, N, N, NB, 14, "ghe", bump=float(N))
    a3 = A3.to_dense_local()
    dp.lauum(ctx, uplo, A3)
    t3 = a3.tril() if uplo == 122 else a3.triu()
    ref = t3.conj().T @ t3 if uplo == 122 else t3 @ t3.conj().T
    sel2 = (lambda x: x.tril()) if uplo == 122 else (lambda x: x.triu())
    assert rel_err(sel2(A3.to_dense_local()), sel2(ref)) < 1e-12


@pytest.mark.parametrize("dtype", [torch.float64, torch.complex128])
def test_potrf_upper_via_lower(monkeypatch, dtype):
    """Upper Cholesky through the transposed lower schedule (one process): same factor as the native
    upper schedule, strictly-lower triangle untouched."""
    import dplasma_amd as dp
    ctx = dp.init(device="cpu")
    N, NB = 300, 64
    A = dp.block_cyclic(ctx, dtype, NB, NB, N, N)
    dp.plghe(ctx, float(N), dp.dplasmaUpperLower, A, 51)
    dense0 = A.to_dense_local().clone()
    B = A.like()
    dp.lacpy(ctx, dp.dplasmaUpperLower, A, B)
    potrf = dp.zpotrf if dtype.is_complex else dp.dpotrf
    monkeypatch.setenv("DPLASMA_POTRF_UPPER", "via_lower")
    assert potrf(ctx, dp.dplasmaUpper, A) == 0
    monkeypatch.setenv("DPLASMA_POTRF_UPPER", "native")
    assert potrf(ctx, dp.dplasmaUpper, B) == 0
    a, b = A.to_dense_local(), B.to_dense_local()
    assert torch.allclose(torch.triu(a), torch.triu(b), atol=1e-10, rtol=1e-10)
    assert torch.equal(torch.tril(a, -1), torch.tril(dense0, -1))
