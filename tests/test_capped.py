"""Memory-capped execution of any tile DAG (runtime/capped.py): host-resident matrices stream through
a bounded tile arena (LRU, write-back), the PaRSEC device memory manager's role for every task class
(tests/Testings.cmake:147 1gpu_lowmem).  CPU: the arena logic with DPLASMA:GPU:number_of_blocks on a CPU
context, results identical to the uncapped run; GPU: host matrices on a GPU context."""
import pytest
import torch

import dplasma_amd as dp


def _ctx(device, nblocks=0):
    ctx = dp.Context(device=device)
    if nblocks:
        ctx.info.set("DPLASMA:GPU:number_of_blocks", str(nblocks))
    return ctx


def _qr(ctx, N, NB, IB=8, dev="cpu"):
    A = dp.TiledMatrix(torch.float64, NB, NB, N, N, device=dev)
    dp.plrnt(dp.Context(device="cpu") if dev == "cpu" else ctx, A, 3872)
    T = dp.TiledMatrix(torch.float64, IB, NB, A.mt * IB, N, device=dev)
    tp = dp.geqrf_New(ctx, A, T)
    tp.execute(ctx)
    return A, T, tp


@pytest.mark.parametrize("nblocks", [4, 9, 40])
def test_geqrf_capped_matches_uncapped_cpu(nblocks):
    A1, T1, tp1 = _qr(_ctx("cpu", nblocks), 96, 16)
    assert tp1.capped.nslots == nblocks
    if nblocks <= 9:
        assert tp1.capped.writebacks > tp1.capped.loads // 4 and tp1.capped.loads > 72   # tiles streamed
    # the same tile DAG without a cap (forced off the stacked-domain engine through the tile format)
    ctx = _ctx("cpu")
    A = dp.TiledMatrix(torch.float64, 16, 16, 96, 96, device="cpu")
    dp.plrnt(ctx, A, 3872)
    T = dp.TiledMatrix(torch.float64, 8, 16, A.mt * 8, 96, device="cpu")
    from dplasma_amd.models import qr
    from dplasma_amd.runtime.dag import TileDAG
    dag = TileDAG(ctx, "geqrf")
    qr._factor(dag, qr._L(A), qr._L(T), qr._L(T), qr._kinds(A, T, False), qr.qrtree.FlatTree(A.mt, A.nt))
    dag.compile().execute(ctx)
    assert torch.equal(A1.data, A.data) and torch.equal(T1.data, T.data)


def test_gels_capped_cpu():
    """Factor + apply (unmqr) + triangular solve, all through the arena."""
    ctx = _ctx("cpu", 6)
    N, NB = 64, 16
    A = dp.TiledMatrix(torch.float64, NB, NB, N, N, device="cpu")
    dp.plrnt(ctx, A, 11)
    a = A.to_dense_local().clone()
    B = dp.TiledMatrix(torch.float64, NB, NB, N, 3, device="cpu")
    dp.plrnt(ctx, B, 12)
    b = B.to_dense_local().clone()
    T = dp.TiledMatrix(torch.float64, 8, NB, A.mt * 8, N, device="cpu")
    dp.geqrf(ctx, A, T)
    dp.geqrs(ctx, A, T, B)
    x = B.to_dense_local()
    assert (a @ x - b).abs().max() < 1e-10


def test_getrf_incpiv_capped_cpu():
    from test_lu_incpiv import _solve
    c1, c0 = _ctx("cpu", 7), _ctx("cpu")
    r1, r0 = _solve(c1, torch.float64, 80, 16, 4), _solve(c0, torch.float64, 80, 16, 4)
    assert r1[0] == 0 and r0[0] == 0
    for i in (1, 2, 4):
        assert torch.equal(r1[i].data, r0[i].data)


def test_dtd_bodies_capped_cpu():
    """DTD task classes (Python bodies on tile views) run on arena views too."""
    from dplasma_amd.models.dtd_potrf import potrf_dtd
    ctx = _ctx("cpu", 5)
    N, NB = 80, 16
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plghe(ctx, float(N), dp.dplasmaUpperLower, A, 8)
    L = torch.linalg.cholesky(A.to_dense_local())
    A2 = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plghe(ctx, float(N), dp.dplasmaUpperLower, A2, 8)
    assert potrf_dtd(ctx, dp.dplasmaLower, A2, window=7) == 0
    assert (torch.tril(A2.to_dense_local()) - L).abs().max() < 1e-10


@pytest.mark.gpu
def test_geqrf_lowmem_gpu():
    """Host matrix and T on a GPU context through 24 device tile slots (QR's 1gpu_lowmem)."""
    ctx = _ctx("cuda:0", 24)
    N, NB = 1024, 128
    A = dp.TiledMatrix(torch.float64, NB, NB, N, N, device="cpu")
    dp.plrnt(dp.Context(device="cpu"), A, 3872)
    a = A.to_dense_local().clone()
    T = dp.TiledMatrix(torch.float64, 32, NB, A.mt * 32, N, device="cpu")
    tp = dp.geqrf_New(ctx, A, T)
    tp.execute(ctx)
    assert tp.capped.loads > 64 and tp.capped.writebacks > 0
    r = torch.triu(A.to_dense_local())
    ref = torch.linalg.qr(a, mode="r")[1]
    assert ((r.abs() - ref.abs()).abs().max() / a.abs().max()) < 1e-10


@pytest.mark.gpu
def test_getrf_incpiv_lowmem_gpu():
    ctx = _ctx("cuda:0", 20)
    N, NB, IB = 768, 96, 32
    A = dp.TiledMatrix(torch.float64, NB, NB, N, N, device="cpu")
    dp.plrnt(dp.Context(device="cpu"), A, 3)
    a = A.to_dense_local().clone()
    B = dp.TiledMatrix(torch.float64, NB, NB, N, 4, device="cpu")
    dp.plrnt(dp.Context(device="cpu"), B, 4)
    b = B.to_dense_local().clone()
    L = dp.incpiv_L_descriptor(ctx, A, IB)        # host-resident like A
    IP = dp.incpiv_ipiv_descriptor(ctx, A)
    assert dp.gesv_incpiv(ctx, A, L, IP, B) == 0
    x = B.to_dense_local()
    assert (a @ x - b).abs().max() / (a.abs().max() * x.abs().max() * N) < 1e-14
