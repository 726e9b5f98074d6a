"""Multi-rank (gloo, CPU) tests: distributed algorithms match the single-rank result."""
import pytest
import torch

from helpers import run_distributed


def _potrf_worker(rank, world, P, N, NB, uplo, prec):
    import dplasma_amd as dp
    ctx = dp.init(device="cpu", P=P)
    dt = dp.PREC_DTYPE[prec]
    A = dp.block_cyclic(ctx, dt, NB, NB, N, N)
    dp.plghe(ctx, float(N), uplo, A, 3872)
    A0 = A.like()
    dp.lacpy(ctx, dp.dplasmaUpperLower, A, A0)
    info = dp.potrf(ctx, uplo, A)
    ok, res = dp.check_potrf(ctx, uplo, A, A0)
    return info, ok, res, A.to_dense_local()


@pytest.mark.parametrize("world,P", [(2, 1), (2, 2), (4, 2), (3, 1), (4, 4)])
@pytest.mark.parametrize("uplo", [122, 121])
def test_potrf_distributed(world, P, uplo):
    N, NB = 150, 19
    out = run_distributed(_potrf_worker, world, P, N, NB, uplo, "d")
    full = sum(out[r][3] for r in range(world))
    for r in range(world):
        info, ok, res, _ = out[r]
        assert info == 0 and ok, (r, res)
    # compare with the single-rank factor
    import dplasma_amd as dp
    ctx = dp.Context(device="cpu")
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plghe(ctx, float(N), uplo, A, 3872)
    dp.potrf(ctx, uplo, A)
    ref = A.to_dense_local()
    tri = (lambda x: x.tril()) if uplo == 122 else (lambda x: x.triu())
    assert (tri(full) - tri(ref)).abs().max() < 1e-12


@pytest.mark.parametrize("world,P", [(2, 1), (4, 2)])
@pytest.mark.parametrize("uplo", [122, 121])
@pytest.mark.parametrize("defer,la", [(2, 1), (3, 1), (2, 2), (1, 2)])
def test_potrf_distributed_deferred(world, P, uplo, defer, la, monkeypatch):
    """Blocks of D panels with aggregated NEXT/REST updates (k = D*NB), on a ragged last tile;
    look-ahead 2 splits the bulk update (NEXT2 / REST2, three panel slabs in flight)."""
    monkeypatch.setenv("DPLASMA_POTRF_LOOKAHEAD", str(la))
    monkeypatch.setenv("DPLASMA_POTRF_DEFER", str(defer))
    monkeypatch.setenv("DPLASMA_POTRF_DEFER_MIN_TILES", "3")
    N, NB = 150, 17
    out = run_distributed(_potrf_worker, world, P, N, NB, uplo, "d")
    full = sum(out[r][3] for r in range(world))
    for r in range(world):
        info, ok, res, _ = out[r]
        assert info == 0 and ok, (r, res)
    import dplasma_amd as dp
    ctx = dp.Context(device="cpu")
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plghe(ctx, float(N), uplo, A, 3872)
    dp.potrf(ctx, uplo, A)
    ref = A.to_dense_local()
    tri = (lambda x: x.tril()) if uplo == 122 else (lambda x: x.triu())
    assert (tri(full) - tri(ref)).abs().max() < 1e-12


def _gemm_worker(rank, world, P, ta, tb, kc):
    import dplasma_amd as dp
    ctx = dp.init(device="cpu", P=P)
    M, N, K, NB = 70, 55, 63, 16
    am, an = (M, K) if ta == 111 else (K, M)
    bm, bn = (K, N) if tb == 111 else (N, K)
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, am, an)
    B = dp.block_cyclic(ctx, torch.float64, NB, NB, bm, bn)
    C = dp.block_cyclic(ctx, torch.float64, NB, NB, M, N)
    dp.plrnt(ctx, A, 3872)
    dp.plrnt(ctx, B, 4674)
    dp.plrnt(ctx, C, 2873)
    dp.gemm(ctx, ta, tb, 0.51, A, B, -0.42, C, kc=kc)
    return C.to_dense_local()


@pytest.mark.parametrize("world,P", [(2, 1), (4, 2)])
@pytest.mark.parametrize("ta,tb", [(111, 111), (112, 111), (111, 112), (112, 112)])
def test_gemm_summa(world, P, ta, tb):
    out = run_distributed(_gemm_worker, world, P, ta, tb, 2)
    full = sum(out[r] for r in range(world))
    import dplasma_amd as dp
    ctx = dp.Context(device="cpu")
    M, N, K, NB = 70, 55, 63, 16
    am, an = (M, K) if ta == 111 else (K, M)
    bm, bn = (K, N) if tb == 111 else (N, K)
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, am, an)
    B = dp.block_cyclic(ctx, torch.float64, NB, NB, bm, bn)
    C = dp.block_cyclic(ctx, torch.float64, NB, NB, M, N)
    dp.plrnt(ctx, A, 3872)
    dp.plrnt(ctx, B, 4674)
    dp.plrnt(ctx, C, 2873)
    a, b, c = A.to_dense_local(), B.to_dense_local(), C.to_dense_local()
    op = lambda x, t: x if t == 111 else x.T
    ref = 0.51 * op(a, ta) @ op(b, tb) - 0.42 * c
    assert (full - ref).abs().max() < 1e-12


def _summa_traffic_worker(rank, world, P):
    import dplasma_amd as dp
    from dplasma_amd.parallel.exchange import ExchangePlan
    ctx = dp.init(device="cpu", P=P)
    A = dp.block_cyclic(ctx, torch.float64, 8, 8, 64, 64)
    needs = {r: [(0, m, n) for m in range(8) for n in range(8)] for r in range(world)}   # everyone needs all
    plan = ExchangePlan(ctx, [A], needs, torch.float64, A.device)
    dp.plrnt(ctx, A, 11)
    buf = plan.new_recv_buffer()
    plan.run(buf)
    own = len(list(A.local_tiles()))
    # no tile is sent to myself; my own tiles sit after the remote ones, copied straight from A
    ok = plan.send_counts[ctx.rank] == 0 and plan.recv_counts[ctx.rank] == 0 and plan.nsend == own * (world - 1)
    ok = ok and plan.nremote == 64 - own
    got = torch.stack([buf[plan.offset(0, m, n): plan.offset(0, m, n) + 64] for m in range(8) for n in range(8)])
    return ok, got


def test_exchange_plan_no_self_traffic():
    """SUMMA / redistribution exchange: locally owned tiles never enter the send slab or the all-to-all."""
    out = run_distributed(_summa_traffic_worker, 4, 2)
    import dplasma_amd as dp
    ctx = dp.Context(device="cpu")
    A = dp.block_cyclic(ctx, torch.float64, 8, 8, 64, 64)
    dp.plrnt(ctx, A, 11)
    ref = torch.stack([A.tile(m, n).T.reshape(-1) for m in range(8) for n in range(8)])
    for r in range(4):
        assert out[r][0]
        assert torch.equal(out[r][1], ref)


def _norm_worker(rank, world, P):
    import dplasma_amd as dp
    ctx = dp.init(device="cpu", P=P)
    A = dp.block_cyclic(ctx, torch.float64, 10, 10, 47, 38)
    dp.plrnt(ctx, A, 7)
    return [dp.lange(ctx, n, A) for n in (dp.dplasmaMaxNorm, dp.dplasmaOneNorm, dp.dplasmaInfNorm,
                                          dp.dplasmaFrobeniusNorm)]


def test_norms_distributed():
    out = run_distributed(_norm_worker, 4, 2)
    import dplasma_amd as dp
    ctx = dp.Context(device="cpu")
    A = dp.block_cyclic(ctx, torch.float64, 10, 10, 47, 38)
    dp.plrnt(ctx, A, 7)
    a = A.to_dense_local()
    ref = [a.abs().max().item(), a.abs().sum(0).max().item(), a.abs().sum(1).max().item(), a.norm().item()]
    for r in range(4):
        for g, e in zip(out[r], ref):
            assert abs(g - e) <= 1e-12 * e


def _blas3_worker(rank, world, P):
    import dplasma_amd as dp
    ctx = dp.init(device="cpu", P=P)
    out = {}
    A = dp.block_cyclic(ctx, torch.float64, 12, 12, 50, 50)
    dp.plghe(ctx, 50.0, dp.dplasmaUpperLower, A, 3)
    for side in (141, 142):
        for uplo in (121, 122):
            for trans in (111, 112):
                B = dp.block_cyclic(ctx, torch.float64, 12, 12, 50, 37 if side == 141 else 50)
                if side == 142:
                    B = dp.block_cyclic(ctx, torch.float64, 12, 12, 37, 50)
                dp.plrnt(ctx, B, 4)
                dp.trsm(ctx, side, uplo, trans, 131, 0.5, A, B)
                out[("trsm", side, uplo, trans)] = B.to_dense_local()
    A2 = dp.block_cyclic(ctx, torch.float64, 12, 12, 50, 50)
    dp.plghe(ctx, 50.0, dp.dplasmaUpperLower, A2, 5)
    dp.poinv(ctx, 122, A2)
    out["poinv"] = A2.to_dense_local()
    C = dp.block_cyclic(ctx, torch.float64, 12, 12, 50, 50)
    dp.plrnt(ctx, C, 6)
    dp.hemm(ctx, 141, 122, 1.0, A, C, 0.0, A2)
    out["hemm"] = A2.to_dense_local()
    return out


def test_blas3_distributed_matches_single():
    res = run_distributed(_blas3_worker, 4, 2)
    single = _blas3_worker(0, 1, 1)
    for key in single:
        full = sum(res[r][key] for r in range(4))
        assert (full - single[key]).abs().max() < 1e-10, key


@pytest.mark.parametrize("world,P", [(2, 1), (2, 2), (4, 2), (8, 2), (3, 1), (4, 4), (6, 2)])
@pytest.mark.parametrize("uplo", [122, 121])
@pytest.mark.parametrize("chunk", [1, 3])
def test_potrf_pipelined(world, P, uplo, chunk, monkeypatch):
    """One panel per step with the critical path pipelined in chunks of tile rows
    (models/potrf_dist.py potrf_pipelined_New): TRSM / urgent exchange / NEXT per chunk, bulk
    exchange for the ranks that do not own the next column; ragged last tile."""
    monkeypatch.setenv("DPLASMA_POTRF_DEFER", "1")
    monkeypatch.setenv("DPLASMA_POTRF_CHUNK", str(chunk))
    N, NB = 170, 17
    out = run_distributed(_potrf_worker, world, P, N, NB, uplo, "d")
    full = sum(out[r][3] for r in range(world))
    for r in range(world):
        info, ok, res, _ = out[r]
        assert info == 0 and ok, (r, res)
    import dplasma_amd as dp
    ctx = dp.Context(device="cpu")
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plghe(ctx, float(N), uplo, A, 3872)
    dp.potrf(ctx, uplo, A)
    tri = (lambda x: x.tril()) if uplo == 122 else (lambda x: x.triu())
    assert (tri(full) - tri(A.to_dense_local())).abs().max() < 1e-12
