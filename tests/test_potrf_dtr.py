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
from dplasma_amd.models import potrf_dtr_dist as DD

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
    seg = D.step_segments(plan.key[plan.hi], plan.order, plan.nt)   # the kernel's per-step FIFO segments
    scur = [int(seg[q]) for q in range(len(seg) - 1)]
    low = [0]

    def take_ticket(force_race):
        # a ticket for a ready head of one of the first 8 segments not handed out (lowest first)
        while low[0] < len(scur) and scur[low[0]] >= seg[low[0] + 1]:
            low[0] += 1
        for q in range(low[0], min(low[0] + 8, len(scur))):
            if scur[q] < seg[q + 1] and (ready(int(hi[scur[q]])) or (force_race and q == low[0])):
                scur[q] += 1
                return scur[q] - 1
        return None
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
            if ticket[wk] is None:
                # a ticket for a ready head (and, rarely, a raced one whose task is not ready yet)
                tk = take_ticket(rng.random() < 0.05)
                if tk is not None:
                    ticket[wk], age[wk] = tk, 0
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
            if all(scur[q] >= seg[q + 1] for q in range(len(scur))) and all(x is None for x in ticket) and \
                    all(cur[li] >= len(lists[li]) for li in range(1, 9)):
                break
            stall += 1
            assert stall < 50, f"schedule stalled: tickets {ticket}, heads {[cur[li] for li in range(9)]}"
        else:
            stall = 0
    assert claimed.all()
    return order


@pytest.mark.parametrize("lo_order", ["column", "panel", "deadline", "rowpipe", "step"])
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


@pytest.mark.parametrize("lo_order", ["column", "panel", "deadline", "rowpipe", "step"])
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


def _emulate_q(plan, A, nb, P=8, seed=0, q=None):
    """The push protocol of k_dtr_q (potrf_dtr.queue_plan): a completed task decrements its successors' pending
    counts and pushes the ones it brings to zero into their class's ring; P workers pop the lowest class (FIFO
    inside a class); completions in random order; numpy math on A as _emulate does."""
    q = q or D.queue_plan(plan)
    rng = np.random.default_rng(seed)
    tasks = plan.tasks
    s = nb // 4
    pend = q["ndeps"].astype(np.int64).copy()
    rings = [[] for _ in range(D.NCLASS)]
    for t in np.nonzero(pend == 0)[0]:   # (the sends of a grid plan are no-ops here: one global matrix)
        rings[q["cls"][t]].append(int(t))
    W = {}

    def blk(i, j, r, c):
        return A[i * nb + r * s: i * nb + (r + 1) * s, j * nb + c * s: j * nb + (c + 1) * s]

    def start(t):
        ty, i, j, k0, r, c, nk = (int(tasks[t][f]) for f in ("type", "i", "j", "k0", "r", "c", "nk"))
        if ty == T_UPD:
            acc = blk(i, j, r, c).copy()
            for k in range(k0, k0 + nk):
                acc -= A[i * nb + r * s: i * nb + (r + 1) * s, k * nb:(k + 1) * nb] @ \
                    A[j * nb + c * s: j * nb + (c + 1) * s, k * nb:(k + 1) * nb].T
            return acc
        if ty == T_TRSM:
            return A[i * nb + r * s: i * nb + (r + 1) * s, k0 * nb:(k0 + 1) * nb] @ W[k0]
        if ty == T_POTRF and r == 0:
            return np.linalg.cholesky(A[k0 * nb:(k0 + 1) * nb, k0 * nb:(k0 + 1) * nb])
        return None

    def finish(t, val):
        ty, i, j, k0, r, c = (int(tasks[t][f]) for f in ("type", "i", "j", "k0", "r", "c"))
        if val is not None:
            if ty == T_UPD:
                if i == j and r == c:
                    val = np.tril(val) + np.triu(blk(i, j, r, c), 1)
                blk(i, j, r, c)[:] = val
            elif ty == T_TRSM:
                A[i * nb + r * s: i * nb + (r + 1) * s, k0 * nb:(k0 + 1) * nb] = val
            else:
                A[k0 * nb:(k0 + 1) * nb, k0 * nb:(k0 + 1) * nb] = np.tril(val)
                W[k0] = np.linalg.inv(val).T
        for x in q["succ"][q["succ_off"][t]:q["succ_off"][t + 1]]:
            pend[x] -= 1
            if pend[x] == 0:
                rings[q["cls"][x]].append(int(x))
    inflight, done = [], 0
    while done < len(tasks):
        while len(inflight) < P:
            ring = next((r_ for r_ in rings if r_), None)
            if ring is None:
                break
            t = ring.pop(0)
            inflight.append((t, start(t)))
        assert inflight, "push protocol stalled"
        t, v = inflight.pop(int(rng.integers(len(inflight))))
        finish(t, v)
        done += 1
    assert (pend == 0).all()


@pytest.mark.parametrize("grid", [(1, 2), (2, 2), (2, 4)])
@pytest.mark.parametrize("nt", [6, 9])
def test_dtr_dist_queue_numerics(grid, nt):
    """Push scheduling over a grid (DistPlan.queue): the cross-rank edges (send -> remote consumers) order every
    task after its inputs -- random completion orders over all ranks' tasks give the factor -- and every rank's
    rings hold exactly its tasks."""
    nb = 16
    n = nt * nb
    rng = np.random.default_rng(5)
    M = rng.standard_normal((n, n))
    S = M @ M.T + n * np.eye(n)
    dplan = DD.DistPlan(nt, 4, *grid)
    q = dplan.queue()
    nring = D.NCLASS * 8
    for r in range(dplan.nranks):
        b = q["qbase"][r * (nring + 1):(r + 1) * (nring + 1)]
        assert b[-1] == q["nown"][r] == int((dplan.owner == r).sum())
    for seed in range(2):
        A = S.copy()
        _emulate_q(dplan, A, nb, P=(16, 48)[seed], seed=seed, q=q)
        assert np.abs(np.tril(A) - np.linalg.cholesky(S)).max() < 1e-10


@pytest.mark.parametrize("lo_order", ["column", "step"])
@pytest.mark.parametrize("nt,defer,min_tiles", [(5, 2, 0), (7, 4, 0), (11, 4, 6)])
def test_dtr_queue_plan_numerics(nt, defer, min_tiles, lo_order):
    """Push scheduling: the requirement lists turned into task edges give the Cholesky factor for random
    completion orders, and every task is pushed exactly once."""
    nb = 16
    n = nt * nb
    rng = np.random.default_rng(7)
    M = rng.standard_normal((n, n))
    S = M @ M.T + n * np.eye(n)
    for seed in range(3):
        A = S.copy()
        plan = D._Plan(nt, defer, lo_order, min_tiles)
        _emulate_q(plan, A, nb, P=(8, 24, 64)[seed], seed=seed)
        assert np.abs(np.tril(A) - np.linalg.cholesky(S)).max() < 1e-10


# ------------------------------------------------------------------------------- distributed DTR
def _emulate_dist(dplan, xcds_of, A=None, nb=None, wpx=2, seed=0):
    """The claim protocol of every rank of a P x Q grid (models/potrf_dtr_dist.py), with wpx workers per
    XCD, random completion order and, with A, per-rank storage: a rank reads its own tiles, its receive
    slots (written only by SEND tasks) and its own W_k (computed by POTRF, or written by SENDW) -- a
    missing requirement shows up as a wrong factor.  Returns the assembled factor (or None)."""
    rng = np.random.default_rng(seed)
    tasks, reqs, nr, nt = dplan.tasks, dplan.reqs, dplan.nranks, dplan.nt
    hi, hi_off, lo, lo_off = dplan.lists(xcds_of)
    cnt = np.zeros((nr, dplan.ncnt), dtype=np.int64)
    segs = dplan.hs_off.reshape(nr, -1)                 # per-rank step segments (relative to hi_off[r])
    scur = [[int(hi_off[r] + segs[r][q]) for q in range(segs.shape[1] - 1)] for r in range(nr)]
    sl = [0] * nr

    def take_ticket(r, force_race):
        end = lambda q: hi_off[r] + segs[r][q + 1]   # noqa: E731
        while sl[r] < len(scur[r]) and scur[r][sl[r]] >= end(sl[r]):
            sl[r] += 1
        for q in range(sl[r], min(sl[r] + 8, len(scur[r]))):
            if scur[r][q] < end(q) and (ready(int(hi[scur[r][q]]), r) or (force_race and q == sl[r])):
                scur[r][q] += 1
                return scur[r][q] - 1
        return None
    hcur = [hi_off[r] for r in range(nr)]
    lcur = [lo_off[x] for x in range(8)]
    s = nb // 4 if nb else None
    store = [A.copy() if A is not None else None for _ in range(nr)]     # rank r's view (its tiles valid)
    if A is not None:
        for r in range(nr):
            for i in range(nt):
                for j in range(nt):
                    if dplan._owner(i, j) != r:
                        store[r][i * nb:(i + 1) * nb, j * nb:(j + 1) * nb] = np.nan
    recv = [dict() for _ in range(nr)]
    W = [dict() for _ in range(nr)]
    workers = [(r, x) for r in range(nr) for x in xcds_of[r] for _ in range(wpx)]
    busy = [False] * len(workers)
    ticket = [None] * len(workers)
    inflight = []
    done = np.zeros(len(tasks), dtype=bool)

    def ready(t, r):
        b, n = tasks["req_beg"][t], tasks["nreq"][t]
        return all(cnt[r, reqs[b + q, 0]] >= reqs[b + q, 1] for q in range(n))

    def panel(r, i, k):
        if dplan._owner(i, k) == r:
            return store[r][i * nb:(i + 1) * nb, k * nb:(k + 1) * nb]
        return recv[r][(i, k)]

    def start(t, r):
        if A is None:
            return None
        tk = tasks[t]
        ty, i, j, k0, rr, c, nk = (int(tk[f]) for f in ("type", "i", "j", "k0", "r", "c", "nk"))
        X = store[r]
        if ty == T_UPD:
            acc = X[i * nb + rr * s: i * nb + (rr + 1) * s, j * nb + c * s: j * nb + (c + 1) * s].copy()
            for k in range(k0, k0 + nk):
                acc -= panel(r, i, k)[rr * s:(rr + 1) * s] @ panel(r, j, k)[c * s:(c + 1) * s].T
            return acc
        if ty == T_TRSM:
            return X[i * nb + rr * s: i * nb + (rr + 1) * s, k0 * nb:(k0 + 1) * nb] @ W[r][k0]
        if ty == T_POTRF and rr == 0:
            return np.linalg.cholesky(X[k0 * nb:(k0 + 1) * nb, k0 * nb:(k0 + 1) * nb])
        if ty == DD.T_SEND:
            return X[i * nb + rr * s: i * nb + (rr + 1) * s, k0 * nb:(k0 + 1) * nb].copy()
        if ty == DD.T_SENDW:
            return W[r][k0][:, rr * s:(rr + 1) * s].copy()
        return None

    def finish(t, r, val):
        tk = tasks[t]
        ty, i, j, k0, rr, c = (int(tk[f]) for f in ("type", "i", "j", "k0", "r", "c"))
        tgt = r
        if A is not None and val is not None:
            X = store[r]
            if ty == T_UPD:
                blk = X[i * nb + rr * s: i * nb + (rr + 1) * s, j * nb + c * s: j * nb + (c + 1) * s]
                if i == j and rr == c:
                    val = np.tril(val) + np.triu(blk, 1)
                blk[:] = val
            elif ty == T_TRSM:
                X[i * nb + rr * s: i * nb + (rr + 1) * s, k0 * nb:(k0 + 1) * nb] = val
            elif ty == T_POTRF:
                X[k0 * nb:(k0 + 1) * nb, k0 * nb:(k0 + 1) * nb] = np.tril(val)
                W[r][k0] = np.linalg.inv(val).T
            elif ty == DD.T_SEND:
                recv[j].setdefault((i, k0), np.full((nb, nb), np.nan))[rr * s:(rr + 1) * s] = val
            else:
                W[j].setdefault(k0, np.zeros((nb, nb)))[:, rr * s:(rr + 1) * s] = val
        if ty in (DD.T_SEND, DD.T_SENDW):
            tgt = j
        if tk["inc"] >= 0:
            cnt[tgt, tk["inc"]] += 1
        done[t] = True

    def try_low(r, x):
        xs = [x] + [y for y in xcds_of[r] if y != x]
        for y in xs:
            if lcur[y] < lo_off[y + 1]:
                t = int(lo[lcur[y]])
                if ready(t, r):
                    lcur[y] += 1
                    return t
                if y == x:
                    return None        # the own head waits: no stealing while the own list lasts
        return None

    stall = 0
    while True:
        progressed = False
        for w in rng.permutation(len(workers)):
            if busy[w]:
                continue
            r, x = workers[w]
            if ticket[w] is None:
                ticket[w] = take_ticket(r, rng.random() < 0.05)
            t = None
            if ticket[w] is not None:
                th = int(hi[ticket[w]])
                if ready(th, r):
                    t, ticket[w] = th, None
            if t is None and (ticket[w] is None or tasks["type"][hi[ticket[w]]] != T_POTRF or stall):
                t = try_low(r, x)
            if t is None:
                continue
            inflight.append((t, r, start(t, r), w))
            busy[w] = True
            progressed = True
        if not progressed and inflight:
            q = int(rng.integers(len(inflight)))
            t, r, v, w = inflight.pop(q)
            busy[w] = False
            finish(t, r, v)
            progressed = True
        if not progressed:
            if all(scur[r][q] >= hi_off[r] + segs[r][q + 1] for r in range(nr) for q in range(len(scur[r]))) and \
                    all(tk is None for tk in ticket) and \
                    all(lcur[y] >= lo_off[y + 1] for y in range(8)):
                break
            stall += 1
            assert stall < 50, f"distributed schedule stalled: heads {hcur} {lcur}"
        else:
            stall = 0
    assert done.all()
    if A is None:
        return None
    L = np.zeros_like(A)
    for i in range(nt):
        for j in range(i + 1):
            o = dplan._owner(i, j)
            L[i * nb:(i + 1) * nb, j * nb:(j + 1) * nb] = store[o][i * nb:(i + 1) * nb, j * nb:(j + 1) * nb]
    return np.tril(L)


def _xcds(nr, mode):
    if mode == "emulate":            # every XCD a rank's GPU: rank r on XCDs [r*8/nr, (r+1)*8/nr)
        X = 8 // nr
        return {r: list(range(r * X, (r + 1) * X)) for r in range(nr)}
    return {r: [r % 8] for r in range(nr)}   # (one list per rank is enough for the protocol check)


@pytest.mark.parametrize("order", ["column", "rowpipe", "step"])
@pytest.mark.parametrize("grid", [(1, 1), (1, 2), (2, 1), (2, 2), (2, 4)])
@pytest.mark.parametrize("nt,defer", [(4, 2), (9, 4), (12, 3)])
def test_dtr_dist_plan_progress(grid, nt, defer, order):
    """Every rank's lists drain with random completion orders: no distributed deadlock."""
    P, Q = grid
    dplan = DD.DistPlan(nt, defer, P, Q, lo_order=order)
    nr = P * Q
    hi, hi_off, lo, lo_off = dplan.lists(_xcds(nr, "emulate"))
    ids = np.concatenate([hi, lo])
    assert len(ids) == len(dplan.tasks) and len(np.unique(ids)) == len(ids)
    # sends exactly to the ranks whose updates read a remote strip, never to the producer itself
    snd = dplan.tasks[dplan.tasks["type"] == DD.T_SEND]
    assert (dplan._owner(snd["i"], snd["k0"]) != snd["j"]).all()
    for seed in range(2):
        _emulate_dist(dplan, _xcds(nr, "emulate"), wpx=1 + seed, seed=seed)


@pytest.mark.parametrize("order", ["column", "rowpipe", "step"])
@pytest.mark.parametrize("grid", [(1, 2), (2, 2), (2, 4), (3, 2)])
def test_dtr_dist_plan_numerics(grid, order):
    """Per-rank storage, receive slots and W copies: the assembled factor equals numpy's Cholesky."""
    P, Q = grid
    nt, nb = 7, 16
    n = nt * nb
    rng = np.random.default_rng(11)
    M = rng.standard_normal((n, n))
    S = M @ M.T + n * np.eye(n)
    dplan = DD.DistPlan(nt, 2, P, Q, lo_order=order)
    nr = P * Q
    L = _emulate_dist(dplan, _xcds(nr, "emulate" if 8 % nr == 0 else "proc"), A=S.copy(), nb=nb, wpx=2, seed=5)
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


@pytest.mark.gpu
@pytest.mark.parametrize("grid", [(1, 2), (2, 2), (2, 4)])
def test_dtr_dist_emulation_gpu(grid):
    """A P x Q grid emulated on the XCDs of one GPU (per-rank storage, sends as copies, dilated time): the
    assembled factor passes the reference residual check."""
    import dplasma_amd as dp
    P, Q = grid
    ctx = dp.init()
    em = DD.Emulation(ctx, 4096, P, Q, bw_gbs=50.0, lat_us=10.0)
    for _ in range(2):
        em.reset()
        em.run()
    L, A0 = em.assemble()
    ok, res = dp.check_potrf(ctx, dp.dplasmaLower, L, A0)
    assert ok, res


def _emulate_q_interleaved(plan, P, seed, skip=True):
    """k_dtr_q's idle-worker protocol at the granularity of its memory operations, in random interleavings: an idle
    worker (1) reads g.done, (2) skips the ring scan when g.done still equals the value read before its last empty scan
    (the scan skip), else scans and pops -- and a completion (a) pushes the successors it readies, then (b) bumps
    g.done.  Returns the number of scheduling steps; raises when every worker idles on a skipped scan while a ring
    holds a task (the deadlock the skip must not introduce)."""
    q = D.queue_plan(plan)
    rng = np.random.default_rng(seed)
    pend = q["ndeps"].astype(np.int64).copy()
    rings = [[] for _ in range(D.NCLASS)]
    for t in np.nonzero(pend == 0)[0]:
        rings[q["cls"][t]].append(int(t))
    done = 0
    # worker: [state, task, dnow, seen]; states: "read" (about to read g.done), "scan", "run", "pushed"
    W = [["read", -1, 0, -1] for _ in range(P)]
    steps = 0
    n = len(plan.tasks)
    while done < n:
        steps += 1
        w = W[int(rng.integers(P))]
        if w[0] == "read":
            w[2] = done
            w[0] = "scan"
        elif w[0] == "scan":
            if skip and w[2] == w[3]:
                w[0] = "read"          # skipped: nothing completed since the last empty scan
            else:
                ring = next((r_ for r_ in rings if r_), None)
                if ring is None:
                    w[3] = w[2]
                    w[0] = "read"
                else:
                    w[1] = ring.pop(0)
                    w[3] = -1
                    w[0] = "run"
        elif w[0] == "run":
            t = w[1]
            for x in q["succ"][q["succ_off"][t]:q["succ_off"][t + 1]]:
                pend[x] -= 1
                if pend[x] == 0:
                    rings[q["cls"][x]].append(int(x))
            w[0] = "pushed"
        else:   # "pushed": the completion's g.done bump, after its pushes
            done += 1
            w[0], w[1] = "read", -1
        if all(x[0] in ("read", "scan") and x[2] == x[3] == done for x in W) and any(rings):
            raise AssertionError("scan skip deadlock: every worker skips while a task is ready")
        if steps > 200 * n * P:
            raise AssertionError("no progress")
    assert (pend == 0).all() and not any(rings)
    return steps


@pytest.mark.parametrize("nt,P", [(6, 4), (9, 16), (12, 64)])
def test_dtr_scan_skip_protocol(nt, P):
    """The idle scan skip (dtr.hip k_dtr_q, one process): a worker skips scanning while g.done has not moved since its
    last empty scan; completions push before they bump g.done -- every task is popped exactly once and no interleaving
    leaves a ready task behind sleeping workers."""
    plan = D._Plan(nt, 4, "column", 0)
    for seed in range(4):
        _emulate_q_interleaved(plan, P, seed)


def test_dtr_plan_disk_cache(tmp_path, monkeypatch):
    """The on-disk plan cache (potrf_dtr._get_plan): a second process-level lookup loads exactly the plan and push
    arrays the first one built; a different planner source or knob misses; DPLASMA_DTR_PLAN_CACHE=0 disables it."""
    monkeypatch.setenv("DPLASMA_DTR_PLAN_CACHE", str(tmp_path))
    D._PLANS.clear()
    p1 = D._get_plan(48, 4, "column", 0, ())
    files = list(tmp_path.iterdir())
    assert len(files) == 1 and files[0].suffix == ".npz"
    D._PLANS.clear()
    p2 = D._get_plan(48, 4, "column", 0, ())
    assert p2 is not p1 and p2.tasks.dtype == p1.tasks.dtype and np.array_equal(p1.tasks, p2.tasks)
    for n in D._PLAN_ARR:
        assert np.array_equal(getattr(p1, n), getattr(p2, n)), n
    assert (p1.nt, p1.S, p1.D, p1.ncnt, p1.WB, p1.order, p1.blocks) == (p2.nt, p2.S, p2.D, p2.ncnt, p2.WB, p2.order,
                                                                        p2.blocks)
    assert set(p1._queue) == set(p2._queue)
    for k, v in p1._queue.items():
        assert np.array_equal(v, p2._queue[k]), k
    monkeypatch.setenv("DPLASMA_DTR_BL_W", "75,65,250,500")   # another priority knob: another file
    assert D._plan_cache_path(48, 4, "column", 0, ()) != str(files[0])
    monkeypatch.setenv("DPLASMA_DTR_PLAN_CACHE", "0")
    assert D._plan_cache_path(48, 4, "column", 0, ()) is None
    D._PLANS.clear()


def test_dtr_scheduler_model_bounds():
    """tools/dtr_sim.py (the CPU model of the push scheduler used to rank priority schemes): every task runs once, no
    task starts before its predecessors end, and the modelled span lies between the DAG's critical path and the
    serial sum of the work."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tools"))
    import dtr_sim as S
    plan = D._Plan(12, 4, "column", 0)
    q = D.queue_plan(plan)
    s, e = S.simulate(plan, q, 32)
    assert (s >= 0).all() and (e >= s).all()
    for t in range(len(plan.tasks)):
        for x in q["succ"][q["succ_off"][t]:q["succ_off"][t + 1]]:
            assert s[x] >= e[t] - 1e-9
    T = plan.tasks
    w = np.where(T["type"] == D.T_UPD, np.where(T["nk"] <= 1, S.DUR["upd1"], S.DUR["upd4_per_k"] * T["nk"]),
                 np.where(T["type"] == D.T_TRSM, S.DUR["trsm"], S.DUR["potrf_blk"]))
    cp = D.bottom_levels(q["succ_off"], q["succ"], w.astype(np.float64)).max()
    assert cp * 0.99 <= e.max() <= (w.sum() + len(T) * 10) * 1.01
