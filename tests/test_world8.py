"""World = 8 (the bench grid, 2 x 4) on CPU gloo ranks: deferred-block POTRF (with the PRI_CHANGE
knob), SUMMA GEMM with look-ahead 1 and 3, and the P x Q partial-pivoting LU (panel all-gather,
look-ahead tasks) -- every result equal to the single-rank one (reference tests/Testings.cmake:171-258
runs the same algorithms on 2-D grids)."""
import os

import numpy as np
import pytest
import torch

from helpers import run_distributed

pytestmark = pytest.mark.slow


def _potrf_w(rank, world, N, NB):
    os.environ["DPLASMA_POTRF_DEFER_MIN_TILES"] = "4"
    os.environ["DPOTRF"] = "3"
    import dplasma_amd as dp
    ctx = dp.init(device="cpu", P=2)
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plghe(ctx, float(N), dp.dplasmaLower, A, 3872)
    A0 = A.like()
    dp.lacpy(ctx, dp.dplasmaUpperLower, A, A0)
    tp = dp.potrf_New(ctx, dp.dplasmaLower, A)
    streams = {t.name: t.stream for t in tp.tasks}
    info = tp.execute(ctx)
    ok, res = dp.check_potrf(ctx, dp.dplasmaLower, A, A0)
    return info, ok, res, A.to_dense_local(), streams


def test_potrf_2x4():
    N, NB = 224, 16
    out = run_distributed(_potrf_w, 8, N, NB)
    full = sum(out[r][3] for r in range(8))
    for r in range(8):
        assert out[r][0] == 0 and out[r][1], out[r][2]
    import dplasma_amd as dp
    ctx = dp.Context(device="cpu")
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plghe(ctx, float(N), dp.dplasmaLower, A, 3872)
    dp.potrf(ctx, dp.dplasmaLower, A)
    assert (full.tril() - A.to_dense_local().tril()).abs().max() < 1e-12
    # DPOTRF=3: the last three panels' critical-path tasks leave the panel stream
    nt = N // NB
    streams = out[0][4]
    assert streams.get(f"POTRF({nt - 1})", "update") == "update"
    assert any(v == "panel" for k, v in streams.items() if k.startswith("NEAR(0)") or k.startswith("POTRF(0)"))


def _gemm_w(rank, world, la):
    import dplasma_amd as dp
    ctx = dp.init(device="cpu", P=2)
    ctx.info.set("DPLASMA:GEMM:look_ahead", str(la))
    M, N, K, NB = 96, 80, 112, 16
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, M, K)
    B = dp.block_cyclic(ctx, torch.float64, NB, NB, K, N)
    C = dp.block_cyclic(ctx, torch.float64, NB, NB, M, N)
    dp.plrnt(ctx, A, 3872)
    dp.plrnt(ctx, B, 4674)
    dp.plrnt(ctx, C, 2873)
    tp = dp.gemm_New(ctx, dp.dplasmaNoTrans, dp.dplasmaNoTrans, 0.51, A, B, -0.42, C, kc=1)
    nbuf = len(tp._buffers)
    tp.execute(ctx)
    return C.to_dense_local(), nbuf


@pytest.mark.parametrize("la", [1, 3])
def test_gemm_summa_2x4_lookahead(la):
    out = run_distributed(_gemm_w, 8, la)
    full = sum(out[r][0] for r in range(8))
    import dplasma_amd as dp
    ctx = dp.Context(device="cpu")
    M, N, K, NB = 96, 80, 112, 16
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, M, K)
    B = dp.block_cyclic(ctx, torch.float64, NB, NB, K, N)
    C = dp.block_cyclic(ctx, torch.float64, NB, NB, M, N)
    dp.plrnt(ctx, A, 3872)
    dp.plrnt(ctx, B, 4674)
    dp.plrnt(ctx, C, 2873)
    ref = 0.51 * A.to_dense_local() @ B.to_dense_local() - 0.42 * C.to_dense_local()
    assert (full - ref).abs().max() < 1e-12
    assert all(out[r][1] == la + 1 for r in range(8))   # one receive buffer per chunk in flight


def _getrf_w(rank, world, N, NB):
    import os
    os.environ["DPLASMA_LU_PANEL"] = "gather"
    import dplasma_amd as dp
    ctx = dp.init(device="cpu", P=2)
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plrnt(ctx, A, 3872)
    IPIV = dp.ptgpanel_ipiv_descriptor(ctx, A)
    tp = dp.getrf_ptgpanel_New(ctx, A, IPIV)
    info = tp.execute(ctx)
    from dplasma_amd.models.lu import _gather_ipiv
    piv = _gather_ipiv(ctx, IPIV)
    st = tp._state
    return info, A.to_dense_local(), piv, list(st.bytes_panel), ctx.mycol


def test_getrf_ptgpanel_2x4():
    N, NB = 160, 16
    out = run_distributed(_getrf_w, 8, N, NB)
    full = sum(out[r][1] for r in range(8))
    import dplasma_amd as dp
    ctx = dp.Context(device="cpu")
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plrnt(ctx, A, 3872)
    IP = dp.ipiv_descriptor(ctx, A)
    assert dp.getrf_1d(ctx, A, IP) == 0
    from dplasma_amd.models.lu import _gather_ipiv
    piv1 = _gather_ipiv(ctx, IP)
    for r in range(8):
        assert out[r][0] == 0
        assert np.array_equal(out[r][2], piv1)          # pivots identical to one process
    assert (full - A.to_dense_local()).abs().max() < 1e-10
    # panel traffic: in the panel's process column each process row sends only its own tiles,
    # i.e. the two process rows of a column together send exactly one panel (not P panels)
    nt = N // NB
    for k in range(nt):
        pc = k % 4
        sent = [out[r][3][k] for r in range(8) if out[r][4] == pc]
        assert sum(sent) == (N - k * NB) * NB, (k, sent)


def _getrf_percol_w(rank, world, N, NB, P, prec):
    import os
    os.environ["DPLASMA_LU_PANEL"] = "percol"
    return _getrf_prec_w(rank, world, N, NB, P, prec)


def _getrf_dist_w(rank, world, N, NB, P, prec):
    import os
    os.environ["DPLASMA_LU_PANEL"] = "dist"
    return _getrf_prec_w(rank, world, N, NB, P, prec)


def _getrf_prec_w(rank, world, N, NB, P, prec):
    import dplasma_amd as dp
    ctx = dp.init(device="cpu", P=P)
    dt = dp.PREC_DTYPE[prec]
    A = dp.block_cyclic(ctx, dt, NB, NB, N, N)
    dp.plrnt(ctx, A, 3872)
    IPIV = dp.ptgpanel_ipiv_descriptor(ctx, A)
    tp = dp.getrf_ptgpanel_New(ctx, A, IPIV)
    info = tp.execute(ctx)
    from dplasma_amd.models.lu import _gather_ipiv
    piv = _gather_ipiv(ctx, IPIV)
    st = tp._state
    return info, A.to_dense_local(), piv, list(st.bytes_panel), ctx.mycol, st.percol


@pytest.mark.parametrize("world,P,prec", [(2, 2, "d"), (4, 2, "d"), (8, 2, "d"), (4, 4, "z"), (2, 1, "d")])
def test_getrf_ptgpanel_percol(world, P, prec):
    """Distributed pivoting (zgetrf_ptgpanel.jdf GETRF_MAX / RDC / SND): every process row keeps its
    own panel rows and each column's pivot comes from one small all-gather of the local candidates.
    Pivots are identical to one process and the per-panel traffic of a rank is O(NB (NB + P))
    elements, independent of M (the gather mode sends M NB / P)."""
    N, NB = 176, 16
    out = run_distributed(_getrf_percol_w, world, N, NB, P, prec)
    import dplasma_amd as dp
    ctx = dp.Context(device="cpu")
    A = dp.block_cyclic(ctx, dp.PREC_DTYPE[prec], NB, NB, N, N)
    dp.plrnt(ctx, A, 3872)
    IP = dp.ipiv_descriptor(ctx, A)
    assert dp.getrf_1d(ctx, A, IP) == 0
    from dplasma_amd.models.lu import _gather_ipiv
    piv1 = _gather_ipiv(ctx, IP)
    full = sum(out[r][1] for r in range(world))
    for r in range(world):
        assert out[r][0] == 0 and out[r][5] == (P > 1)
        assert np.array_equal(out[r][2], piv1)
    assert (full - A.to_dense_local()).abs().max() < 1e-10
    if P > 1:
        Q = world // P
        nt = N // NB
        for k in range(nt):
            sent = [out[r][3][k] for r in range(world) if out[r][4] == k % Q]
            assert max(sent) == NB * (2 + 2 * NB), (k, sent)          # per column: value, row, 2 rows
            if N - k * NB > P * (2 * NB + 2):                        # tall panels: less than gathering
                assert max(sent) < (N - k * NB) * NB // P


@pytest.mark.parametrize("world,P,prec", [(2, 2, "d"), (4, 2, "d"), (8, 4, "d"), (4, 4, "z"), (3, 3, "s"), (2, 1, "d")])
def test_getrf_ptgpanel_dist(world, P, prec):
    """Distributed-pivoting P > 1 panel (ops.lu_dist_ops, zgetrf_ptgpanel.jdf GETRF_MAX / RDC / SND): every process
    row keeps its own panel rows plus a replica of the diagonal tile; each column's pivot and the
    winner's whole row travel in one exchange of P candidates.  Pivots are identical to one process;
    a rank sends kmin x (2 + NB) elements to each of its P - 1 peers per panel, independent of M."""
    N, NB = 176, 16
    out = run_distributed(_getrf_dist_w, world, N, NB, P, prec)
    import dplasma_amd as dp
    ctx = dp.Context(device="cpu")
    A = dp.block_cyclic(ctx, dp.PREC_DTYPE[prec], NB, NB, N, N)
    dp.plrnt(ctx, A, 3872)
    IP = dp.ipiv_descriptor(ctx, A)
    assert dp.getrf_1d(ctx, A, IP) == 0
    from dplasma_amd.models.lu import _gather_ipiv
    piv1 = _gather_ipiv(ctx, IP)
    full = sum(out[r][1] for r in range(world))
    for r in range(world):
        assert out[r][0] == 0
        assert np.array_equal(out[r][2], piv1)
    tol = 1e-3 if prec in ("s", "c") else 1e-10
    assert (full - A.to_dense_local()).abs().max() < tol
    if P > 1:
        Q = world // P
        for k in range(N // NB):
            sent = [out[r][3][k] for r in range(world) if out[r][4] == k % Q]
            assert max(sent) == NB * (2 + NB) * (P - 1), (k, sent)
