"""DTD insert-task front end: generic bodies, hazards, distribution, and the DTD Cholesky."""
import pytest
import torch

import dplasma_amd as dp
from dplasma_amd.models.dtd_potrf import potrf_dtd
from dplasma_amd.runtime import dtd
from helpers import rel_err, run_distributed


@pytest.fixture(scope="module")
def ctx():
    return dp.init(device="cpu")


def test_dtd_program_order_semantics(ctx):
    """A chain of read/write tasks on shared tiles must observe program order (RAW/WAR/WAW)."""
    A = dp.block_cyclic(ctx, torch.float64, 4, 4, 8, 8)
    tp = dtd.taskpool_new(ctx)
    T = dtd.tile_of

    def setv(a, v):
        a.fill_(v)

    def axpy(x, y, alpha):  # y += alpha * x
        y.add_(alpha * x)
    tp.insert_task(setv, (T(A, 0, 0), dtd.OUTPUT), 1.0)
    tp.insert_task(setv, (T(A, 1, 1), dtd.OUTPUT), 2.0)
    tp.insert_task(axpy, (T(A, 0, 0), dtd.INPUT), (T(A, 1, 1), dtd.INOUT), 3.0)   # A11 = 2 + 3 = 5
    tp.insert_task(setv, (T(A, 0, 0), dtd.OUTPUT), 7.0)                            # WAR on A00
    tp.insert_task(axpy, (T(A, 1, 1), dtd.INPUT), (T(A, 0, 0), dtd.INOUT), 1.0)   # A00 = 7 + 5 = 12
    tp.execute()
    a = A.to_dense_local()
    assert (a[:4, :4] == 12).all() and (a[4:, 4:] == 5).all()


@pytest.mark.parametrize("uplo", [dp.dplasmaLower, dp.dplasmaUpper])
@pytest.mark.parametrize("dt", [torch.float64, torch.complex128])
def test_potrf_dtd(ctx, uplo, dt):
    N, NB = 70, 16
    A = dp.block_cyclic(ctx, dt, NB, NB, N, N)
    dp.plghe(ctx, float(N), dp.dplasmaUpperLower, A, 3)
    a = A.to_dense_local()
    assert potrf_dtd(ctx, uplo, A) == 0
    L = torch.linalg.cholesky(a)
    got = A.to_dense_local()
    if uplo == dp.dplasmaLower:
        assert rel_err(torch.tril(got), L) < 1e-12
    else:
        assert rel_err(torch.triu(got), L.conj().T) < 1e-12


@pytest.mark.parametrize("window", [1, 7, 40])
def test_potrf_dtd_windows_overlap_insertion(ctx, window):
    """Windowed DTD: windows launch while insertion continues (windows_run grows with the task
    count), data_flush keeps at most KEEP windows of remote copies, the result is unchanged."""
    N, NB = 90, 16
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plghe(ctx, float(N), dp.dplasmaUpperLower, A, 5)
    L = torch.linalg.cholesky(A.to_dense_local())
    assert potrf_dtd(ctx, dp.dplasmaLower, A, window=window) == 0
    tp = potrf_dtd.last
    assert tp.windows_run >= tp.ntasks // window // 2 and tp.windows_run > 1
    assert len(tp._live) == 0
    assert rel_err(torch.tril(A.to_dense_local()), L) < 1e-12


def test_potrf_dtd_untied(ctx):
    """One inserted task inserts the whole factorisation from its body (testing_zpotrf_dtd_untied.c)."""
    from dplasma_amd.models.dtd_potrf import potrf_dtd_untied
    N, NB = 80, 16
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plghe(ctx, float(N), dp.dplasmaUpperLower, A, 8)
    L = torch.linalg.cholesky(A.to_dense_local())
    assert potrf_dtd_untied(ctx, dp.dplasmaLower, A, window=9) == 0
    assert potrf_dtd_untied.last.ntasks > 1 and potrf_dtd_untied.last.windows_run > 2
    assert rel_err(torch.tril(A.to_dense_local()), L) < 1e-12


@pytest.mark.parametrize("ta,tb", [(111, 111), (112, 111), (111, 113)])
def test_gemm_dtd(ctx, ta, tb):
    """tests/testing_zgemm_dtd.c: GEMM through insert_task matches the dense product."""
    from dplasma_amd.models.dtd_potrf import gemm_dtd
    M, N, K, NB = 50, 40, 36, 8
    dt = torch.complex128 if tb == 113 else torch.float64
    A = dp.block_cyclic(ctx, dt, NB, NB, *((M, K) if ta == 111 else (K, M)))
    B = dp.block_cyclic(ctx, dt, NB, NB, *((K, N) if tb == 111 else (N, K)))
    C = dp.block_cyclic(ctx, dt, NB, NB, M, N)
    for X, s in ((A, 1), (B, 2), (C, 3)):
        dp.plrnt(ctx, X, s)
    a, b, c = A.to_dense_local(), B.to_dense_local(), C.to_dense_local()
    op = lambda x, t: x if t == 111 else (x.T if t == 112 else x.conj().T)  # noqa: E731
    gemm_dtd(ctx, ta, tb, 0.5, A, B, -0.25, C, window=13)
    assert rel_err(C.to_dense_local(), 0.5 * op(a, ta) @ op(b, tb) - 0.25 * c) < 1e-12


def _worker(rank, world, P, window=None):
    import dplasma_amd as dp
    from dplasma_amd.models.dtd_potrf import potrf_dtd
    ctx = dp.init(device="cpu", P=P)
    A = dp.block_cyclic(ctx, torch.float64, 16, 16, 70, 70)
    dp.plghe(ctx, 70.0, dp.dplasmaUpperLower, A, 3)
    return potrf_dtd(ctx, dp.dplasmaLower, A, window=window), A.to_dense_local()


@pytest.mark.parametrize("world,P,window", [(2, 1, None), (4, 2, None), (4, 2, 11)])
def test_potrf_dtd_distributed(world, P, window):
    out = run_distributed(_worker, world, P, window)
    ctx = dp.init(device="cpu")
    A = dp.block_cyclic(ctx, torch.float64, 16, 16, 70, 70)
    dp.plghe(ctx, 70.0, dp.dplasmaUpperLower, A, 3)
    L = torch.linalg.cholesky(A.to_dense_local())
    assert all(out[r][0] == 0 for r in range(world))
    assert rel_err(torch.tril(sum(out[r][1] for r in range(world))), L) < 1e-12


def _untied_worker(rank, world, P, uplo, window):
    import dplasma_amd as dp
    from dplasma_amd.models.dtd_potrf import potrf_dtd_untied
    ctx = dp.init(device="cpu", P=P)
    A = dp.block_cyclic(ctx, torch.float64, 16, 16, 70, 70)
    dp.plghe(ctx, 70.0, dp.dplasmaUpperLower, A, 3)
    info = potrf_dtd_untied(ctx, uplo, A, window=window)
    return info, A.to_dense_local(), potrf_dtd_untied.last.windows_run


@pytest.mark.parametrize("world,P,uplo,window", [(2, 2, 122, 12), (4, 2, 121, 20), (4, 1, 122, None)])
def test_potrf_dtd_untied_distributed(world, P, uplo, window):
    """testing_zpotrf_dtd_untied.c on several processes: the inserter task has no data, runs on every rank
    and returns AGAIN whenever the window is nearly full; every rank inserts the same tasks."""
    out = run_distributed(_untied_worker, world, P, uplo, window)
    ctx = dp.init(device="cpu")
    A = dp.block_cyclic(ctx, torch.float64, 16, 16, 70, 70)
    dp.plghe(ctx, 70.0, dp.dplasmaUpperLower, A, 3)
    L = torch.linalg.cholesky(A.to_dense_local())
    assert all(out[r][0] == 0 for r in range(world))
    full = sum(out[r][1] for r in range(world))
    got = torch.tril(full) if uplo == 122 else torch.triu(full).T
    assert rel_err(got, L) < 1e-12
    if window:
        assert all(out[r][2] > 3 for r in range(world))   # AGAIN re-entered the inserter several times


def test_dtd_dataless_task_runs_everywhere_with_again(ctx):
    """A task without tile arguments runs where it is inserted; AGAIN calls it again after a launch."""
    from dplasma_amd.runtime import dtd
    tp = dtd.taskpool_new(ctx, "t", window=4)
    A = dp.block_cyclic(ctx, torch.float64, 4, 4, 16, 16)
    calls = []

    def inc(a):
        a.add_(1.0)

    def inserter(state):
        calls.append(tp.windows_run)
        while state[0] < 10:
            tp.insert_task(inc, (dtd.tile_of(A, state[0] % 4, 0), dtd.INOUT))
            state[0] += 1
            if tp.pending >= 3:
                return dtd.AGAIN
        return None
    tp.insert_task(tp.task_class("ins", inserter), [0])
    tp.wait()
    assert len(calls) == 4 and calls[0] == 0 and calls[-1] >= 3
    assert float(A.tile(0, 0).sum()) == 3 * 16 and float(A.tile(1, 0).sum()) == 3 * 16


@pytest.mark.gpu
def test_gpu_potrf_dtd():
    g = dp.init(device="cuda:0")
    N, NB = 1000, 128
    A = dp.block_cyclic(g, torch.float64, NB, NB, N, N)
    dp.plghe(g, float(N), dp.dplasmaUpperLower, A, 3)
    a = A.to_dense_local().cpu()
    assert potrf_dtd(g, dp.dplasmaLower, A) == 0
    assert rel_err(torch.tril(A.to_dense_local().cpu()), torch.linalg.cholesky(a)) < 1e-11


def test_dtd_priority_orders_ready_tasks(ctx):
    """insert_task(priority=...) (tests/testing_zpotrf_dtd.c passes one on every insert): tasks that
    are ready together run highest priority first; program order breaks ties, and dependencies
    still win over priorities."""
    A = dp.block_cyclic(ctx, torch.float64, 2, 2, 12, 12)
    T = dtd.tile_of
    order = []

    def mark(a, tag):
        order.append(tag)
        a.fill_(float(len(order)))

    tp = dtd.taskpool_new(ctx, window=0)
    prios = [0, 5, 1, 5, -2, 3]
    for i, p in enumerate(prios):
        tp.insert_task(mark, (T(A, i, i), dtd.INOUT), i, priority=p)
    # a dependent low-priority-then-high chain on one tile: order must stay RAW
    tp.insert_task(mark, (T(A, 0, 1), dtd.INOUT), "dep0", priority=-9)
    tp.insert_task(mark, (T(A, 0, 1), dtd.INOUT), "dep1", priority=99)
    tp.compile().execute(ctx)
    first = [t for t in order if isinstance(t, int) or t == "dep0"]
    # level 0: the six diagonal tasks and dep0, by priority (ties in program order)
    assert first == [1, 3, 5, 2, 0, 4, "dep0"]
    assert order.index("dep1") > order.index("dep0")

    # without priorities: program order
    order.clear()
    tp = dtd.taskpool_new(ctx, window=0)
    for i in range(6):
        tp.insert_task(mark, (T(A, i, i), dtd.INOUT), i)
    tp.compile().execute(ctx)
    assert order == list(range(6))
