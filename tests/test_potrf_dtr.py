"""Device task runtime Cholesky (models/potrf_dtr.py + csrc/kernels/dtr.hip).

CPU: the task table is checked by an emulator of the kernel's claim protocol -- a high-priority list
and eight per-XCD low lists, a list head claimed only when its (counter, target) requirements hold,
counters bumped at completion, up to P tasks in flight completing in random order -- which must
(a) never stall (deadlock freedom of the list orders), (b) claim every task once, and (c) computing
each task's tile math in numpy at claim / completion time, reproduce numpy's Cholesky.
GPU: the persistent kernel against the CPU fp64 reference of the same factorisation.
"""
import numpy as np
import pytest
import torch

from dplasma_amd.models import potrf_dtr as D

T_UPD, T_TRSM, T_POTRF = D.T_UPD, D.T_TRSM, D.T_POTRF


def _emulate(plan, A=None, nb=None, P=8, seed=0, steal=False):
    """Run the plan's claim protocol with P workers and random completion order; optional numpy math on A
    (lower, nt x nt tiles of nb, sub-tiles of nb / 4).  Returns the claim order."""
    rng = np.random.default_rng(seed)
    tasks, reqs = plan.tasks, plan.reqs
    cnt = np.zeros(plan.ncnt, dtype=np.int64)
    lists = [plan.hi] + [plan.lo[plan.lo_off[x]:plan.lo_off[x + 1]] for x in range(8)]
    cur = [0] * 9
    inflight = []    # (task, start value, worker)
    claimed = np.zeros(len(tasks), dtype=bool)
    order = []
    s = nb // 4 if nb else None
    W = {}

    def ready(t):
        b, n = tasks["req_beg"][t], tasks["nreq"][t]
        return all(cnt[reqs[b + q, 0]] >= reqs[b + q, 1] for q in range(n))

    def blk(i, j, r, c):
        return A[i * nb + r * s: i * nb + (r + 1) * s, j * nb + c * s: j * nb + (c + 1) * s]

    def start(t):
        tk = tasks[t]
        if A is None:
            return None
        ty, i, j, k0, r, c, nk = (int(tk[f]) for f in ("type", "i", "j", "k0", "r", "c", "nk"))
        if ty == T_UPD:
            acc = blk(i, j, r, c).copy()
            for k in range(k0, k0 + nk):
                acc -= A[i * nb + r * s: i * nb + (r + 1) * s, k * nb:(k + 1) * nb] @ \
                    A[j * nb + c * s: j * nb + (c + 1) * s, k * nb:(k + 1) * nb].T
            return acc
        if ty == T_TRSM:
            Wk = W[k0]
            return A[i * nb + r * s: i * nb + (r + 1) * s, k0 * nb:(k0 + 1) * nb] @ Wk
        if ty == T_POTRF and r == 0:
            L = np.linalg.cholesky(A[k0 * nb:(k0 + 1) * nb, k0 * nb:(k0 + 1) * nb])
            return L
        return None

    def finish(t, val):
        tk = tasks[t]
        if A is not None and val is not None:
            ty, i, j, k0, r, c = (int(tk[f]) for f in ("type", "i", "j", "k0", "r", "c"))
            if ty == T_UPD:
                if i == j and r == c:
                    val = np.tril(val) + np.triu(blk(i, j, r, c), 1)
                blk(i, j, r, c)[:] = val
            elif ty == T_TRSM:
                A[i * nb + r * s: i * nb + (r + 1) * s, k0 * nb:(k0 + 1) * nb] = val
            else:
                A[k0 * nb:(k0 + 1) * nb, k0 * nb:(k0 + 1) * nb] = np.tril(val)
                W[k0] = np.linalg.inv(val).T
        if tk["inc"] >= 0:
            cnt[tk["inc"]] += 1

    # the kernel's claim protocol: high list by ticket (in order, taken when the head is ready; a holder
    # whose task is not ready yet helps with ready low-list heads -- a POTRF holder only after a while),
    # low lists per XCD
    # (own list first, another XCD's only once the own one is exhausted)
    hi = lists[0]
    hcur = 0
    ticket = [None] * P
    age = [0] * P
    busy = [False] * P
    owner = {}
    stall = 0

    def try_low(wk):
        # steal=True (the kernel's DtrArgs.flags bit 0): another XCD's ready head also when the own head
        # waits on a dependency, not only once the own list is exhausted
        x = wk % 8
        own_done = cur[1 + x] >= len(lists[1 + x])
        order = [x] + ([(x + d) % 8 for d in range(1, 8)] if (own_done or steal) else [])
        for xx in order:
            li = 1 + xx
            lst = lists[li]
            if cur[li] < len(lst) and ready(lst[cur[li]]):
                t = int(lst[cur[li]])
                cur[li] += 1
                return t
        return None

    while True:
        progressed = False
        for wk in rng.permutation(P):
            if busy[wk]:
                continue
            if ticket[wk] is None and hcur < len(hi) and (ready(int(hi[hcur])) or rng.random() < 0.05):
                # a ticket for a ready head (and, rarely, a raced one whose task is not ready yet)
                ticket[wk], age[wk] = hcur, 0
                hcur += 1
            t = None
            if ticket[wk] is not None:
                th = int(hi[ticket[wk]])
                if ready(th):
                    t, ticket[wk] = th, None
                else:
                    age[wk] += 1
            if t is None and (ticket[wk] is None or tasks["type"][hi[ticket[wk]]] != T_POTRF or age[wk] > 3
                              or stall):
                t = try_low(wk)
            if t is None:
                continue
            claimed[t] = True
            order.append(t)
            inflight.append((t, start(t), wk))
            busy[wk] = True
            progressed = True
        if not progressed and inflight:
            q = int(rng.integers(len(inflight)))
            t, v, wk = inflight.pop(q)
            busy[wk] = False
            finish(t, v)
            progressed = True
        if not progressed:
            if hcur >= len(hi) and all(x is None for x in ticket) and all(cur[li] >= len(lists[li]) for li in range(1, 9)):
                break
            stall += 1
            assert stall < 50, f"schedule stalled: tickets {ticket}, heads {[cur[li] for li in range(9)]}"
        else:
            stall = 0
    assert claimed.all()
    return order


@pytest.mark.parametrize("lo_order", ["column", "panel"])
@pytest.mark.parametrize("nt,defer", [(1, 4), (3, 4), (9, 4), (12, 2), (10, 3)])
def test_dtr_plan_lists_and_progress(nt, defer, lo_order):
    plan = D._Plan(nt, defer, lo_order)
    ids = np.concatenate([plan.hi, plan.lo])
    assert len(ids) == len(plan.tasks) and len(np.unique(ids)) == len(ids)
    assert (plan.tasks["nreq"] <= 10).all()
    n_potrf = (plan.tasks["type"] == T_POTRF).sum()
    assert n_potrf == 16 * nt
    for seed in range(3):
        _emulate(plan, P=(8, 13, 40)[seed], seed=seed)   # >= 1 worker per XCD, as the kernel's grid has
        _emulate(plan, P=(8, 13, 40)[seed], seed=seed, steal=True)


@pytest.mark.parametrize("lo_order", ["column", "panel"])
@pytest.mark.parametrize("nt,defer,min_tiles", [(5, 2, 0), (7, 4, 0), (11, 4, 6)])
def test_dtr_plan_numerics(nt, defer, min_tiles, lo_order):
    nb = 16
    n = nt * nb
    rng = np.random.default_rng(7)
    M = rng.standard_normal((n, n))
    S = M @ M.T + n * np.eye(n)
    A = S.copy()
    plan = D._Plan(nt, defer, lo_order, min_tiles)
    _emulate(plan, A=A, nb=nb, P=8, seed=3, steal=(lo_order == "panel"))
    L = np.tril(A)
    assert np.abs(L - np.linalg.cholesky(S)).max() < 1e-10


@pytest.mark.gpu
@pytest.mark.parametrize("N", [512, 2048, 5120])
def test_dtr_potrf_gpu(N):
    import dplasma_amd as dp
    ctx = dp.init()
    A = dp.block_cyclic(ctx, torch.float64, 512, 512, N, N)
    dp.dplghe(ctx, float(N), dp.dplasmaLower, A, 3872)
    A0 = A.data.clone()
    tp = D.potrf_dtr_New(ctx, dp.dplasmaLower, A)
    for rep in range(2):          # the same taskpool twice: per-launch epochs / counter reset
        A.data.copy_(A0)
        info = tp.execute(ctx)
        assert info == 0
    Ar = A.like()
    Ar.data.copy_(A0)
    ok, res = dp.check_potrf(ctx, dp.dplasmaLower, A, Ar)
    assert ok, res
