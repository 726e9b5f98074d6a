"""CU-reserved critical-path streams (DPLASMA_DIAG_CUS, context._reserve_cus): POTRF uses its own
masked "diag" / "potrf_update" streams, every other algorithm keeps the unmasked shared streams (the
persistent grid-barrier panel kernels of LU / QR size their grids for every CU), and the masked
streams are destroyed by Context.release()."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def masked_ctx(monkeypatch):
    monkeypatch.setenv("DPLASMA_DIAG_CUS", "16")
    import dplasma_amd as dp
    ctx = dp.Context(device="cuda:0")
    assert "diag" in ctx.streams and "potrf_update" in ctx.streams
    yield ctx
    ctx.release()
    assert "diag" not in ctx.streams and not ctx._owned_streams


def test_potrf_on_masked_streams(masked_ctx):
    import dplasma_amd as dp
    N, NB = 4096, 512
    A = dp.block_cyclic(masked_ctx, torch.float64, NB, NB, N, N)
    dp.dplghe(masked_ctx, float(N), dp.dplasmaLower, A, 3872)
    A0 = A.like()
    dp.lacpy(masked_ctx, dp.dplasmaUpperLower, A, A0)
    tp = dp.dpotrf_New(masked_ctx, dp.dplasmaLower, A)
    assert any(t.stream == "diag" for t in tp.tasks)
    assert tp.execute(masked_ctx) == 0
    ok, res = dp.check_potrf(masked_ctx, dp.dplasmaLower, A, A0)
    assert ok, res


def test_getrf_keeps_unmasked_streams(masked_ctx):
    import dplasma_amd as dp
    N, NB = 2048, 256
    A = dp.block_cyclic(masked_ctx, torch.float64, NB, NB, N, N)
    dp.plrnt(masked_ctx, A, 3872)
    a = A.to_dense_local().cpu()
    IP = dp.ipiv_descriptor(masked_ctx, A)
    tp = dp.getrf_1d_New(masked_ctx, A, IP)
    assert all(t.stream in ("panel", "update", "aux") for t in tp.tasks)
    assert tp.execute(masked_ctx) == 0
    lu = A.to_dense_local().cpu()
    L = torch.tril(lu, -1) + torch.eye(N, dtype=torch.float64)
    piv = IP.to_dense_local().view(-1).cpu().long() - 1
    perm = torch.arange(N)
    for i, p in enumerate(piv.tolist()):
        perm[[i, p]] = perm[[p, i]]
    assert ((L @ torch.triu(lu) - a[perm]).abs().max() / a.abs().max()).item() < 1e-12
