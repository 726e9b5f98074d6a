"""Memory-bounded GEMM with host-resident operands (src/zgemm_NN_gpu.jdf; the reference's
``lowmem`` GPU tests force eviction with a tiny device memory budget -- here the block
sizes are forced small through the DPLASMA:GEMM:GPU:{b,c,d} info keys)."""
import pytest
import torch

import dplasma_amd as dp
from helpers import DTYPES

T = (dp.dplasmaNoTrans, dp.dplasmaTrans, dp.dplasmaConjTrans)


def test_gemm_gpu_requires_gpu_context():
    ctx = dp.init(device="cpu")
    A = dp.block_cyclic(ctx, torch.float64, 8, 8, 16, 16)
    with pytest.raises(ValueError):
        dp.gemm_gpu_New(ctx, T[0], T[0], 1.0, A, A, 0.0, A)


def _host(ctx, dt, m, n, nb, seed):
    X = dp.TiledMatrix(dt, nb, nb, m, n, device="cpu")
    dp.plrnt(dp.init(device="cpu"), X, seed)
    return X


@pytest.mark.gpu
@pytest.mark.parametrize("prec", list("dz"))
@pytest.mark.parametrize("ta,tb", [(0, 0), (1, 0), (0, 2), (2, 1)])
def test_gpu_gemm_host_operands(prec, ta, tb):
    dt = DTYPES[prec]
    if not dt.is_complex and 2 in (ta, tb):
        ta, tb = min(ta, 1), min(tb, 1)
    M, N, K, NB = 700, 520, 610, 96
    g = dp.init(device="cuda:0")
    A = _host(g, dt, *((M, K) if ta == 0 else (K, M)), NB, 1)
    B = _host(g, dt, *((K, N) if tb == 0 else (N, K)), NB, 2)
    C = _host(g, dt, M, N, NB, 3)
    a, b, c = (X.to_dense_local() for X in (A, B, C))
    op = lambda x, t: x if t == 0 else (x.t() if t == 1 else x.conj().t())  # noqa: E731
    ref = 0.5 * op(a, ta) @ op(b, tb) - 2.0 * c
    inf = dp.info_create()
    for k, v in (("b", "2"), ("c", "3"), ("d", "2")):
        dp.info_set(inf, "DPLASMA:GEMM:GPU:" + k, v)
    dp.gemm_gpu(g, T[ta], T[tb], 0.5, A, B, -2.0, C, info=inf)
    assert (C.to_dense_local() - ref).abs().max() < 1e-12 * K * ref.abs().max()


@pytest.mark.gpu
def test_gpu_gemm_dispatches_host_operands():
    g = dp.init(device="cuda:0")
    A, B, C = (_host(g, torch.float64, 512, 512, 128, s) for s in (4, 5, 6))
    ref = A.to_dense_local() @ B.to_dense_local()
    tp = dp.gemm_New(g, T[0], T[0], 1.0, A, B, 0.0, C)
    assert tp.name == "gemm_gpu"
    tp.execute(g)
    assert (C.to_dense_local() - ref).abs().max() < 1e-11


def _dist_ooc_worker(rank, world, P, ta, tb, bcd):
    import dplasma_amd as dp
    ctx = dp.init(device="cpu", P=P)
    for key, v in zip(("b", "c", "d"), bcd):
        ctx.info.set(f"DPLASMA:GEMM:GPU:{key}", v)
    M, N, K, NB = 70, 52, 61, 8
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, *((M, K) if ta == 0 else (K, M)))
    B = dp.block_cyclic(ctx, torch.float64, NB, NB, *((K, N) if tb == 0 else (N, K)))
    C = dp.block_cyclic(ctx, torch.float64, NB, NB, M, N)
    for X, s in ((A, 1), (B, 2), (C, 3)):
        dp.plrnt(ctx, X, s)
    tp = dp.gemm_gpu_New(ctx, T[ta], T[tb], 0.5, A, B, -2.0, C, allow_cpu=True)
    tp.execute(ctx)
    return C.to_dense_local(), tp.bytes_recv


@pytest.mark.parametrize("world,P,ta,tb,bcd", [(4, 2, 0, 0, (3, 2, 2)), (4, 2, 1, 0, (2, 4, 3)), (2, 1, 0, 1, (4, 3, 1)),
                                               (3, 3, 1, 1, (5, 5, 4))])
def test_gemm_ooc_distributed(world, P, ta, tb, bcd):
    """Host-resident operands on a P x Q grid (zgemm_NN_gpu.jdf's super-blocks with GLOBAL barriers):
    global b x c blocks of C, K in chunks of d tiles, only the tiles other ranks own are exchanged."""
    from helpers import run_distributed
    out = run_distributed(_dist_ooc_worker, world, P, ta, tb, bcd)
    ctx = dp.init(device="cpu")
    M, N, K, NB = 70, 52, 61, 8
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, *((M, K) if ta == 0 else (K, M)))
    B = dp.block_cyclic(ctx, torch.float64, NB, NB, *((K, N) if tb == 0 else (N, K)))
    C = dp.block_cyclic(ctx, torch.float64, NB, NB, M, N)
    for X, s in ((A, 1), (B, 2), (C, 3)):
        dp.plrnt(ctx, X, s)
    op = lambda x, t: x if t == 0 else x.t()  # noqa: E731
    ref = 0.5 * op(A.to_dense_local(), ta) @ op(B.to_dense_local(), tb) - 2.0 * C.to_dense_local()
    full = sum(out[r][0] for r in range(world))
    assert (full - ref).abs().max() < 1e-10
    assert all(out[r][1] > 0 for r in range(world))   # every rank received remote operand tiles
