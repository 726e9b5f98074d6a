"""Native ready-queue list scheduler (csrc/runtime/dag_core.h list_schedule) behind the reference's
-o scheduler choice: every policy yields a topological order with the policy's tie-breaking, and
algorithms give the same results under every policy."""
import numpy as np
import pytest
import torch

import dplasma_amd as dp
from dplasma_amd.runtime.dag import _lib_rt
from dplasma_amd.runtime.taskpool import SCHED_POLICY, Taskpool, policy_code
from helpers import rel_err

rt = _lib_rt()
pytestmark = pytest.mark.skipif(rt is None, reason="native runtime module not built")


def _csr(preds):
    ptr = np.cumsum([0] + [len(p) for p in preds]).astype(np.int64)
    idx = np.array([d for p in preds for d in p], dtype=np.int64)
    return ptr, idx


def _topo(order, preds):
    pos = {t: i for i, t in enumerate(order)}
    return sorted(order) == list(range(len(preds))) and all(pos[d] < pos[t] for t, p in enumerate(preds) for d in p)


def test_policies_on_a_diamond():
    # 0 -> {1 (prio 1), 2 (prio 5), 3 (prio 3)} -> 4
    preds = [[], [0], [0], [0], [1, 2, 3]]
    prio = np.array([0, 1, 5, 3, 0], dtype=np.int32)
    ptr, idx = _csr(preds)
    sched = lambda pol, seed=0: list(rt.dag_list_schedule(ptr, idx, prio, pol, seed))  # noqa: E731
    assert sched(0) == [0, 1, 2, 3, 4]          # program order
    assert sched(1) == [0, 2, 3, 1, 4]          # priority first
    assert sched(2) == [0, 1, 3, 2, 4]          # inverse priority
    assert sched(3) == [0, 1, 2, 3, 4]          # FIFO of readiness
    assert sched(4) == [0, 3, 2, 1, 4]          # LIFO: last readied first
    for seed in range(5):
        assert _topo(sched(5, seed), preds)


def test_random_dags_every_policy_topological():
    g = np.random.default_rng(1)
    for trial in range(20):
        n = int(g.integers(2, 60))
        preds = [sorted(set(int(x) for x in g.integers(0, t, size=int(g.integers(0, 4))))) if t else []
                 for t in range(n)]
        prio = g.integers(-5, 6, size=n).astype(np.int32)
        ptr, idx = _csr(preds)
        for pol in range(6):
            assert _topo(list(rt.dag_list_schedule(ptr, idx, prio, pol, trial)), preds)


def test_cycle_and_bad_input_rejected():
    ptr, idx = _csr([[1], [0]])
    with pytest.raises(ValueError):
        rt.dag_list_schedule(ptr, idx, np.zeros(2, np.int32), 1, 0)
    with pytest.raises(ValueError):
        rt.dag_list_schedule(np.array([0, 1], np.int64), np.array([7], np.int64), np.zeros(1, np.int32), 1, 0)
    with pytest.raises(ValueError):
        policy_code("nope")


def test_taskpool_issue_order_follows_policy():
    ctx = dp.init(device="cpu")
    log = []
    tp = Taskpool("t", ctx)
    a = tp.task("a", "update", lambda: log.append("a"))
    tp.task("lo", "update", lambda: log.append("lo"), [a], prio=1)
    tp.task("hi", "update", lambda: log.append("hi"), [a], prio=9)
    ctx.scheduler = "ap"
    tp.execute(ctx)
    assert log == ["a", "hi", "lo"]
    log.clear()
    ctx.scheduler = None
    tp.execute(ctx)
    assert log == ["a", "lo", "hi"]


@pytest.mark.parametrize("sched", sorted(k for k in SCHED_POLICY if k))
def test_algorithms_under_every_policy(sched):
    ctx = dp.init(device="cpu")
    ctx.scheduler, ctx.sched_seed = sched, 3
    N, NB = 120, 16
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plghe(ctx, float(N), dp.dplasmaUpperLower, A, 4)
    a = A.to_dense_local()
    import os
    os.environ["DPLASMA_POTRF_DEFER_MIN_TILES"] = "3"
    try:
        assert dp.potrf(ctx, dp.dplasmaLower, A) == 0
    finally:
        del os.environ["DPLASMA_POTRF_DEFER_MIN_TILES"]
    assert rel_err(torch.tril(A.to_dense_local()), torch.linalg.cholesky(a)) < 1e-12
    B = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plrnt(ctx, B, 5)
    b = B.to_dense_local()
    IP = dp.ipiv_descriptor(ctx, B)
    assert dp.getrf_1d(ctx, B, IP) == 0
    lu = B.to_dense_local()
    L = torch.tril(lu, -1) + torch.eye(N, dtype=torch.float64)
    piv = IP.to_dense_local().view(-1).long() - 1
    perm = torch.arange(N)
    for i, p in enumerate(piv.tolist()):
        perm[[i, p]] = perm[[p, i]]
    assert rel_err(L @ torch.triu(lu), b[perm]) < 1e-12


def _potrf_sched_worker(rank, world, P, sched):
    import dplasma_amd as dp
    ctx = dp.init(device="cpu", P=P)
    ctx.scheduler = sched
    N, NB = 170, 17
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
    dp.plghe(ctx, float(N), dp.dplasmaLower, A, 3872)
    tp = dp.potrf_New(ctx, dp.dplasmaLower, A)
    order = tp.issue_order(ctx)
    moved = order != list(range(len(tp.tasks)))
    comm_order = [t for t in order if tp.tasks[t].comm is not False]
    info = tp.execute(ctx)
    return info, A.to_dense_local(), moved, comm_order == sorted(comm_order)


@pytest.mark.parametrize("sched", ["pbq", "ip", "rnd"])
def test_multirank_potrf_under_policy(sched, monkeypatch):
    """On more than one rank a scheduler policy reorders the compute-only tasks (comm=False) while
    the communicating tasks keep their program order on every rank; the factor is bit-identical to
    the program-order run (reference -o choice, tests/common.c:291-314)."""
    from helpers import run_distributed
    monkeypatch.setenv("DPLASMA_POTRF_DEFER_MIN_TILES", "3")
    ref = run_distributed(_potrf_sched_worker, 4, 2, None)
    out = run_distributed(_potrf_sched_worker, 4, 2, sched)
    assert any(out[r][2] for r in range(4)), "the policy never changed the issue order"
    for r in range(4):
        assert out[r][0] == 0 and out[r][3]
        assert torch.equal(out[r][1], ref[r][1]), r
