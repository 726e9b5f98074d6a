"""Complex MFMA GEMM (csrc/kernels/zgemm.hip) against a plain PyTorch complex reference: every
op(A)/op(B) combination (N, T, C), ragged sizes, alpha/beta complex, triangular C masks, several
k-tiles per item, and the generic FMA kernel as a second opinion."""
import pytest
import torch

from dplasma_amd.constants import dplasmaConjTrans, dplasmaNoTrans, dplasmaTrans

pytestmark = pytest.mark.gpu
OPS = [dplasmaNoTrans, dplasmaTrans, dplasmaConjTrans]


def _op(x, t):
    return x if t == dplasmaNoTrans else (x.T if t == dplasmaTrans else x.conj().T)


@pytest.mark.parametrize("dt", [torch.complex128, torch.complex64])
@pytest.mark.parametrize("ta", OPS)
@pytest.mark.parametrize("tb", OPS)
def test_cgemm_ops(dt, ta, tb):
    from dplasma_amd.ops import tile_ops as ops
    from dplasma_amd.ops.batch import GemmBatch
    g = torch.Generator(device="cpu").manual_seed(ta * 7 + tb)
    M, N, K1, K2 = 150, 97, 70, 33
    lda = 211
    def rnd(r, c):
        return torch.randn(r, c, dtype=dt, generator=g)
    # two k-tiles per item: C = beta C + alpha (opA1 opB1 + opA2 opB2)
    A1, A2 = (rnd(M, K1), rnd(M, K2)) if ta == dplasmaNoTrans else (rnd(K1, M), rnd(K2, M))
    B1, B2 = (rnd(K1, N), rnd(K2, N)) if tb == dplasmaNoTrans else (rnd(N, K1), rnd(N, K2))
    C0 = rnd(M, N)
    alpha, beta = complex(0.7, -0.3), complex(-0.4, 0.2)
    store = torch.zeros(lda * 1200, dtype=dt)
    offs = {}
    pos = 0
    for name, X in (("A1", A1), ("A2", A2), ("B1", B1), ("B2", B2), ("C", C0)):
        torch.as_strided(store, X.shape, (1, lda), pos).copy_(X)
        offs[name] = pos
        pos += lda * X.shape[1]
    dev = store.cuda()
    ref = beta * C0 + alpha * (_op(A1, ta) @ _op(B1, tb) + _op(A2, ta) @ _op(B2, tb))
    gb = GemmBatch()
    gb.add(offs["C"], M, N, [(offs["A1"], offs["B1"], K1), (offs["A2"], offs["B2"], K2)])
    gb.finalize()
    for generic in (False, True):
        d = dev.clone()
        old = ops.FORCE_GENERIC_GEMM
        ops.FORCE_GENERIC_GEMM = generic
        try:
            ops.gemm(ta, tb, alpha, d, lda, d, lda, beta, d, lda, gb)
        finally:
            ops.FORCE_GENERIC_GEMM = old
        got = torch.as_strided(d.cpu(), (M, N), (1, lda), offs["C"])
        tol = 1e-12 if dt == torch.complex128 else 2e-4
        assert (got - ref).abs().max().item() / ref.abs().max().item() < tol, generic


@pytest.mark.parametrize("mask", [1, 2])
def test_zgemm_triangle_mask(mask):
    from dplasma_amd.ops import tile_ops as ops
    from dplasma_amd.ops.batch import GemmBatch
    n, k = 130, 40
    A = torch.randn(n, k, dtype=torch.complex128)
    C0 = torch.randn(n, n, dtype=torch.complex128)
    store = torch.cat([A.T.reshape(-1), C0.T.reshape(-1)]).cuda()
    gb = GemmBatch()
    gb.add(n * k, n, n, [(0, 0, k)], mask)
    gb.finalize()
    ops.gemm(dplasmaNoTrans, dplasmaConjTrans, -1.0, store, n, store, n, 1.0, store, n, gb)
    got = store[n * k:].cpu().view(n, n).T
    full = C0 - A @ A.conj().T
    keep = torch.ones(n, n, dtype=torch.bool).tril() if mask == 1 else torch.ones(n, n, dtype=torch.bool).triu()
    exp = torch.where(keep, full, C0)
    assert (got - exp).abs().max().item() < 1e-12
