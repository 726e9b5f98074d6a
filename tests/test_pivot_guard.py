"""Out-of-range pivots reach the row-interchange kernels as an info code, never as a fault or a silent skip.

Every row-move path validates its pivots before moving anything (csrc/kernels/lu_piv.hip
report_bad_pivot; the CPU path of ops/tile_ops.py mirrors it): a pivot outside [i, m) leaves the
matrix untouched and sets info to ops.BAD_PIVOT (-1001) over 0 or a positive singular-column index.
The user-facing laswp / getrs return the same code.  (Reference: a stale or corrupt IPIV reaching
CORE_zlaswp is undefined behaviour there; here it is a reported failure.)"""
import pytest
import torch

import dplasma_amd as dp
from dplasma_amd.models import lu
from dplasma_amd.ops import _lib
from dplasma_amd.ops import tile_ops as ops
from helpers import DTYPES

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _dev(d):
    if d == "cuda":
        _lib.load()
    return d


@pytest.mark.parametrize("dev", DEVICES)
@pytest.mark.parametrize("seg", [(0, 64), (100, 700)])   # net-moves kernel / sequential kernel (> 512 swaps)
@pytest.mark.parametrize("bad", ["high", "negative", "below_i"])
def test_laswp_panel_bad_pivot(dev, seg, bad):
    _dev(dev)
    i0, i1 = seg
    m, ld, ncols = 1000, 1008, 9
    ipiv = torch.tensor([min(m - 1, i + (i % 3)) for i in range(i1)], dtype=torch.int32)
    j = i0 + (i1 - i0) // 2
    ipiv[j] = {"high": m + 5, "negative": -3, "below_i": j - 1}[bad]
    P = torch.randn(ld * (ncols + 2), dtype=torch.float64, device=dev)
    P0 = P.clone()
    for start in (0, 7):   # info over 0 and over a positive (singular column) index
        info = torch.tensor([start], dtype=torch.int32, device=dev)
        ops.laswp_panel(P, ld, 1, 1 + ncols, ipiv.to(dev), i0, i1, m=m, info=info)
        if dev == "cuda":
            torch.cuda.synchronize()
        assert int(info[0]) == ops.BAD_PIVOT
        assert torch.equal(P.cpu(), P0.cpu())   # nothing moved


@pytest.mark.parametrize("dev", DEVICES)
def test_laswp_panel_keeps_other_failure(dev):
    """A pivot failure never overwrites another negative code (e.g. -1000, a panel spin timeout)."""
    _dev(dev)
    ld, m = 64, 60
    ipiv = torch.tensor([70] * 4, dtype=torch.int32, device=dev)
    P = torch.zeros(ld * 4, dtype=torch.float64, device=dev)
    info = torch.tensor([-1000], dtype=torch.int32, device=dev)
    ops.laswp_panel(P, ld, 0, 4, ipiv, 0, 4, m=m, info=info)
    assert int(info[0]) == -1000


@pytest.mark.parametrize("dev", DEVICES)
def test_piv_moves_and_permute_bad_pivot(dev):
    _dev(dev)
    kb, mrel = 16, 40
    ipiv = torch.arange(kb, dtype=torch.int32) + 1
    ipiv[5] = mrel + 2                                  # past the rows below the panel
    dst = torch.zeros(2 * kb, dtype=torch.int32, device=dev)
    src = torch.zeros_like(dst)
    cnt = torch.full((1,), 99, dtype=torch.int32, device=dev)
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    ops.piv_moves(ipiv.to(dev), kb, dst, src, cnt, mrel=mrel, info=info)
    assert int(cnt[0]) == 0 and int(info[0]) == ops.BAD_PIVOT
    # a corrupt move list (a row outside the view) handed to the in-place permutation directly
    mb, nb, nrt = 8, 8, 5
    A = torch.randn(mb * nrt * nb * 2, dtype=torch.float64, device=dev)
    A0 = A.clone()
    rowoff = torch.tensor([t * mb for t in range(nrt)], dtype=torch.int64, device=dev)
    coloff = torch.tensor([0, mb * nrt * nb], dtype=torch.int64, device=dev)
    ncols = torch.tensor([nb, nb], dtype=torch.int32, device=dev)
    d = torch.tensor([0, mb * nrt + 3], dtype=torch.int32, device=dev)
    s_ = torch.tensor([mb * nrt + 3, 0], dtype=torch.int32, device=dev)
    c2 = torch.tensor([2], dtype=torch.int32, device=dev)
    info2 = torch.zeros(1, dtype=torch.int32, device=dev)
    ops.rows_permute(A, mb * nrt, mb, 0, rowoff, coloff, ncols, nb, d, s_, c2, 2, info2)
    if dev == "cuda":
        torch.cuda.synchronize()
    assert int(info2[0]) == ops.BAD_PIVOT
    assert torch.equal(A.cpu(), A0.cpu())


@pytest.mark.parametrize("dev", DEVICES)
def test_getrs_corrupt_ipiv_reports(dev):
    """getrs with a corrupted IPIV returns BAD_PIVOT and leaves B unchanged (both transposes)."""
    _dev(dev)
    ctx = dp.init(device=dev if dev == "cpu" else "cuda:0")
    N, NB = 64, 16
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plrnt(ctx, A, 3)
    IPIV = dp.block_cyclic(ctx, torch.int32, NB, NB, 1, N)
    assert lu.getrf_1d(ctx, A, IPIV) == 0
    for (m, n) in IPIV.local_tiles():
        t = IPIV.tile(m, n)
        if n == 1:
            t[0, 3] = N + 10                     # 1-based pivot past the last row
    B = dp.block_cyclic(ctx, torch.float64, NB, NB, N, 2)
    dp.plrnt(ctx, B, 5)
    b0 = B.to_dense_local()
    for trans in (dp.dplasmaNoTrans, dp.dplasmaTrans):
        assert lu.getrs(ctx, trans, A, IPIV, B) == ops.BAD_PIVOT
        assert torch.equal(B.to_dense_local().cpu(), b0.cpu())
