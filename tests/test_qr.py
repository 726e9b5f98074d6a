"""QR / LQ family: factorizations, Q generation/application, least squares.

Checks follow the reference's testing_zgeqrf.c:221-303 (||I - Q^H Q|| and
||A - Q R|| / ||A||) and testing_zgels.c; the GPU variants compare the HIP
kernels against the CPU reference path of the same algorithm.
"""
import pytest
import torch

import dplasma_amd as dp
from dplasma_amd.models import qr_panel
from helpers import DTYPES, rel_err, run_distributed

EPS = {"s": 1e-5, "c": 1e-5, "d": 1e-13, "z": 1e-13}


def _mk(ctx, dt, M, N, NB, seed, **kw):
    A = dp.block_cyclic(ctx, dt, NB, NB, M, N, **kw)
    dp.plrnt(ctx, A, seed)
    return A


def _T(ctx, A, ib):
    return dp.block_cyclic(ctx, A.dtype, ib, A.nb, A.mt * ib, A.nt * A.nb)


def _qr_check(ctx, prec, M, N, NB, IB, lq=False):
    dt = DTYPES[prec]
    A = _mk(ctx, dt, M, N, NB, 3872)
    a = A.to_dense_local().cpu()
    T = _T(ctx, A, IB)
    K = min(M, N)
    if not lq:
        dp.geqrf(ctx, A, T)
        Q = dp.block_cyclic(ctx, dt, NB, NB, M, K)
        dp.ungqr(ctx, A, T, Q)
        q = Q.to_dense_local().cpu()
        r = torch.triu(A.to_dense_local().cpu()[:K])
        orth = (q.conj().T @ q - torch.eye(K, dtype=dt)).abs().max().item()
        rec = (q @ r - a).abs().max().item() / a.abs().max().item()
    else:
        dp.gelqf(ctx, A, T)
        Q = dp.block_cyclic(ctx, dt, NB, NB, K, N)
        dp.unglq(ctx, A, T, Q)
        q = Q.to_dense_local().cpu()
        l_ = torch.tril(A.to_dense_local().cpu()[:, :K])
        orth = (q @ q.conj().T - torch.eye(K, dtype=dt)).abs().max().item()
        rec = (l_ @ q - a).abs().max().item() / a.abs().max().item()
    lim = EPS[prec] * max(M, N)
    assert orth < lim, orth
    assert rec < lim, rec
    return A, T


@pytest.fixture(scope="module")
def ctx():
    return dp.init(device="cpu")


@pytest.mark.parametrize("prec", list("sdcz"))
@pytest.mark.parametrize("shape", [(40, 24, 8, 4), (37, 23, 8, 3), (30, 30, 10, 4)])
def test_geqrf(ctx, prec, shape):
    _qr_check(ctx, prec, *shape)


@pytest.mark.parametrize("prec", list("dz"))
@pytest.mark.parametrize("shape", [(24, 40, 8, 4), (23, 37, 8, 3)])
def test_gelqf(ctx, prec, shape):
    _qr_check(ctx, prec, *shape, lq=True)


def _dense_q(ctx, A, T, lq):
    """Full square orthogonal factor Q (M x M for QR, N x N for LQ)."""
    n = A.m if not lq else A.n
    Q = dp.block_cyclic(ctx, A.dtype, A.mb, A.nb, n, n)
    (dp.unglq if lq else dp.ungqr)(ctx, A, T, Q)
    return Q.to_dense_local().cpu()


@pytest.mark.parametrize("prec", list("dz"))
@pytest.mark.parametrize("lq", [False, True])
def test_unmqr_unmlq_variants(ctx, prec, lq):
    dt = DTYPES[prec]
    M, N, NB, IB = (36, 20, 8, 4) if not lq else (20, 36, 8, 4)
    A = _mk(ctx, dt, M, N, NB, 11)
    T = _T(ctx, A, IB)
    (dp.gelqf if lq else dp.geqrf)(ctx, A, T)
    q = _dense_q(ctx, A, T, lq)
    n = q.shape[0]
    for side in (dp.dplasmaLeft, dp.dplasmaRight):
        for trans in (dp.dplasmaNoTrans, dp.dplasmaConjTrans):
            shp = (n, 13) if side == dp.dplasmaLeft else (13, n)
            C = _mk(ctx, dt, shp[0], shp[1], NB, 5)
            c = C.to_dense_local().cpu()
            (dp.unmlq if lq else dp.unmqr)(ctx, side, trans, A, T, C)
            op = q if trans == dp.dplasmaNoTrans else q.conj().T
            ref = op @ c if side == dp.dplasmaLeft else c @ op
            assert rel_err(C.to_dense_local().cpu(), ref) < 1e-12, (side, trans)


@pytest.mark.parametrize("prec", list("dz"))
def test_gels_overdetermined(ctx, prec):
    dt = DTYPES[prec]
    M, N, NB, IB, NRHS = 45, 21, 8, 4, 5
    A = _mk(ctx, dt, M, N, NB, 1)
    a = A.to_dense_local()
    B = _mk(ctx, dt, M, NRHS, NB, 2)
    b = B.to_dense_local()
    T = _T(ctx, A, IB)
    dp.gels(ctx, dp.dplasmaNoTrans, A, T, B)
    x = B.to_dense_local()[:N]
    ref = torch.linalg.lstsq(a, b).solution
    assert rel_err(x, ref) < 1e-11


@pytest.mark.parametrize("prec", list("dz"))
def test_gels_underdetermined(ctx, prec):
    dt = DTYPES[prec]
    M, N, NB, IB, NRHS = 19, 42, 8, 4, 3
    A = _mk(ctx, dt, M, N, NB, 1)
    a = A.to_dense_local()
    B = _mk(ctx, dt, N, NRHS, NB, 2)
    b = B.to_dense_local()[:M]
    T = _T(ctx, A, IB)
    dp.gels(ctx, dp.dplasmaNoTrans, A, T, B)
    x = B.to_dense_local()
    ref = torch.linalg.pinv(a) @ b  # minimum-norm solution
    assert rel_err(x, ref) < 1e-11


def test_dag_levels_native_matches_python():
    import numpy as np
    from dplasma_amd.runtime import dag as D
    rt = D._lib_rt()
    rng = np.random.default_rng(0)
    ops = rng.integers(0, 12, size=(300, 3)).astype(np.int64)
    modes = rng.integers(0, 4, size=(300, 3)).astype(np.uint8)
    lp = D._levels_py(ops, modes)
    vp = D._versions_py(ops, modes)
    if rt is not None:
        assert (rt.dag_levels(ops, modes) == lp).all()
        assert (rt.dag_versions(ops, modes) == vp).all()
    # every hazard is respected: a writer is strictly after every earlier access of its tiles
    last = {}
    for t in range(len(ops)):
        for k, md in zip(ops[t], modes[t]):
            if not md:
                continue
            for (pl, pm) in last.get(k, []):
                if (md & 2) or (pm & 2):
                    assert lp[t] > pl
        for k, md in zip(ops[t], modes[t]):
            if md:
                last.setdefault(k, []).append((lp[t], md))


# ----------------------------------------------------------------------------- distributed
def _qr_worker(rank, world, P, lq):
    import dplasma_amd as dp
    ctx = dp.init(device="cpu", P=P)
    dt = torch.float64
    M, N, NB, IB = (44, 28, 8, 4) if not lq else (28, 44, 8, 4)
    A = dp.block_cyclic(ctx, dt, NB, NB, M, N)
    dp.plrnt(ctx, A, 3872)
    T = dp.block_cyclic(ctx, dt, IB, NB, A.mt * IB, A.nt * NB)
    (dp.gelqf if lq else dp.geqrf)(ctx, A, T)
    K = min(M, N)
    Q = dp.block_cyclic(ctx, dt, NB, NB, M if not lq else K, K if not lq else N)
    (dp.unglq if lq else dp.ungqr)(ctx, A, T, Q)
    C = dp.block_cyclic(ctx, dt, NB, NB, M if not lq else N, 9)
    dp.plrnt(ctx, C, 17)
    (dp.unmlq if lq else dp.unmqr)(ctx, dp.dplasmaLeft, dp.dplasmaConjTrans, A, T, C)
    return A.to_dense_local(), T.to_dense_local(), Q.to_dense_local(), C.to_dense_local()


@pytest.mark.parametrize("world,P,lq", [(2, 1, False), (2, 2, False), (4, 2, False), (3, 3, True), (4, 2, True)])
def test_qr_distributed(world, P, lq):
    out = run_distributed(_qr_worker, world, P, lq)
    # single-process run of the same algorithm on the same data: 1 x Q grids take the
    # stacked-domain engine (real QR), P > 1 grids the tile algorithm
    with qr_panel.engine("panel" if P == 1 else "tile"):
        r = _qr_worker(0, 1, 1, lq)
    for i in range(4):
        full = sum(out[k][i] for k in range(world))
        assert rel_err(full, r[i]) < 1e-12, i


# ----------------------------------------------------------------------------- GPU (HIP kernels)
@pytest.fixture(scope="module")
def gctx():
    return dp.init(device="cuda:0")


def _dense(M):
    return M.to_dense_local().cpu()


@pytest.mark.gpu
@pytest.mark.parametrize("prec", list("sdcz"))
@pytest.mark.parametrize("lq", [False, True])
def test_gpu_qr_matches_cpu(gctx, ctx, prec, lq):
    """Same algorithm on GPU (HIP kernels) and CPU (reference path): factors must agree."""
    dt = DTYPES[prec]
    M, N, NB, IB = (200, 136, 32, 8) if not lq else (136, 200, 32, 8)
    out = []
    for c in (gctx, ctx):
        A = _mk(c, dt, M, N, NB, 3872)
        T = _T(c, A, IB)
        (dp.gelqf if lq else dp.geqrf)(c, A, T)
        out.append((_dense(A), _dense(T)))
    tol_ = 1e-4 if prec in "sc" else 1e-11
    assert rel_err(out[0][0], out[1][0]) < tol_
    assert rel_err(out[0][1], out[1][1]) < tol_ * 10


@pytest.mark.gpu
@pytest.mark.parametrize("prec", list("dz"))
@pytest.mark.parametrize("shape", [(520, 300, 64, 16), (300, 300, 96, 32), (256, 512, 64, 32)])
def test_gpu_qr_orthogonality(gctx, prec, shape):
    M, N, NB, IB = shape
    _qr_check(gctx, prec, M, N, NB, IB, lq=M < N)


@pytest.mark.gpu
@pytest.mark.parametrize("lq", [False, True])
def test_gpu_unmqr_variants(gctx, lq):
    dt = torch.complex128
    M, N, NB, IB = (160, 96, 32, 8) if not lq else (96, 160, 32, 8)
    A = _mk(gctx, dt, M, N, NB, 11)
    T = _T(gctx, A, IB)
    (dp.gelqf if lq else dp.geqrf)(gctx, A, T)
    q = _dense_q(gctx, A, T, lq)
    n = q.shape[0]
    for side in (dp.dplasmaLeft, dp.dplasmaRight):
        for trans in (dp.dplasmaNoTrans, dp.dplasmaConjTrans):
            shp = (n, 40) if side == dp.dplasmaLeft else (40, n)
            C = _mk(gctx, dt, shp[0], shp[1], NB, 5)
            c = _dense(C)
            (dp.unmlq if lq else dp.unmqr)(gctx, side, trans, A, T, C)
            op = q if trans == dp.dplasmaNoTrans else q.conj().T
            ref = op @ c if side == dp.dplasmaLeft else c @ op
            assert rel_err(_dense(C), ref) < 1e-12, (side, trans)


@pytest.mark.gpu
def test_gpu_gels(gctx):
    dt = torch.float64
    for (M, N) in ((300, 170), (170, 300)):
        A = _mk(gctx, dt, M, N, 64, 1)
        a = _dense(A)
        B = _mk(gctx, dt, max(M, N), 7, 64, 2)
        b = _dense(B)[:M]
        T = _T(gctx, A, 16)
        dp.gels(gctx, dp.dplasmaNoTrans, A, T, B)
        x = _dense(B)[:N]
        ref = torch.linalg.lstsq(a, b).solution if M >= N else torch.linalg.pinv(a) @ b
        assert rel_err(x, ref) < 1e-10


# ----------------------------------------------------------------------------- QR trees / HQR
def test_qrtree_validity_sweep():
    """Exhaustive sweep of tree parameters (tests/TestsQRPivgen.cmake analogue)."""
    import itertools
    from dplasma_amd.models import qrtree as Q
    for mt, nt in ((7, 4), (12, 12), (5, 9), (16, 3), (1, 1)):
        for ll, hl, a, p, dom, rr in itertools.product(range(5), range(5), (1, 2, 3, 8), (1, 2, 3), (0, 1), (0, 1)):
            Q.HQRTree(mt, nt, ll, hl, a, p, dom, rr).check()
        for p, q in itertools.product((1, 2, 3), (1, 2, 4)):
            Q.SystolicTree(mt, nt, p, q).check()
        Q.SVDTree(mt, nt, 1, 2, 4, 1).check()
        Q.FlatTree(mt, nt).check()


def test_qrtree_queries():
    from dplasma_amd.models import qrtree as Q
    t = Q.HQRTree(8, 4, Q.GREEDY_TREE, Q.FLAT_TREE, a=2, p=2)
    k = 0
    assert t.getnbgeqrf(k) == len(t.heads(k))
    for i in range(t.getnbgeqrf(k)):
        assert t.geti(k, t.getm(k, i)) == i
    for m in range(1, 8):
        p = t.currpiv(k, m)
        # m appears in p's kill sequence, walkable with nextpiv / prevpiv
        seq, x = [], t.nextpiv(k, p, t.mt)
        while x != t.mt:
            seq.append(x)
            x = t.nextpiv(k, p, x)
        assert m in seq
        back, x = [], t.prevpiv(k, p, p)
        while x != t.mt:
            back.append(x)
            x = t.prevpiv(k, p, x)
        assert back[::-1] == seq
    assert t.gettype(0, 2) == Q.KILLED_BY_TS and t.gettype(0, 1) == Q.KILLED_BY_DISTTREE
    # systolic matches the reference's closed forms (dplasma_systolic_qr.c:56-99)
    s = Q.SystolicTree(10, 10, p=2, q=2)
    for k in range(10):
        for m in range(k + 1, 10):
            exp_t = 0 if m >= k + 4 else (1 if m >= k + 2 else 3)
            exp_p = (m - k) % 4 + k if exp_t == 0 else ((m - k) % 2 + k if exp_t == 1 else k)
            assert s.gettype(k, m) == exp_t and s.currpiv(k, m) == exp_p
    assert Q.HQRTree(32, 4, Q.BINARY_TREE, Q.BINARY_TREE, 1, 1).depth(0) < Q.FlatTree(32, 4).depth(0)


def _hqr_run(c, dt, lq, treeargs, M, N, NB, IB):
    A = _mk(c, dt, M, N, NB, 77)
    a = _dense(A)
    TS = _T(c, A, IB)
    TT = _T(c, A, IB)
    tree = dp.hqr_init(dp.dplasmaConjTrans if lq else dp.dplasmaNoTrans, A, *treeargs)
    (dp.gelqf_param if lq else dp.geqrf_param)(c, tree, A, TS, TT)
    K = min(M, N)
    Qm = dp.block_cyclic(c, dt, NB, NB, M if not lq else K, K if not lq else N)
    (dp.unglq_param if lq else dp.ungqr_param)(c, tree, A, TS, TT, Qm)
    q = _dense(Qm)
    if not lq:
        r = torch.triu(_dense(A)[:K])
        e1 = (q.conj().T @ q - torch.eye(K, dtype=dt)).abs().max().item()
        e2 = (q @ r - a).abs().max().item() / a.abs().max().item()
    else:
        l_ = torch.tril(_dense(A)[:, :K])
        e1 = (q @ q.conj().T - torch.eye(K, dtype=dt)).abs().max().item()
        e2 = (l_ @ q - a).abs().max().item() / a.abs().max().item()
    return e1, e2, A, tree, TS, TT


@pytest.mark.parametrize("prec", list("dz"))
@pytest.mark.parametrize("lq", [False, True])
@pytest.mark.parametrize("treeargs", [(1, 0, 2, 3), (3, 3, 1, 2), (2, 1, 3, 2, True), (0, 4, 2, 2, False, True)])
def test_hqr(ctx, prec, lq, treeargs):
    M, N = (70, 40) if not lq else (40, 70)
    e1, e2, *_ = _hqr_run(ctx, DTYPES[prec], lq, treeargs, M, N, 8, 4)
    assert e1 < 1e-13 and e2 < 1e-13


def test_hqr_unmqr_and_solve(ctx):
    dt = torch.float64
    e1, e2, A, tree, TS, TT = _hqr_run(ctx, dt, False, (1, 3, 2, 2), 60, 30, 8, 4)
    B = _mk(ctx, dt, 60, 4, 8, 9)
    b = _dense(B)
    A2 = _mk(ctx, dt, 60, 30, 8, 77)
    dp.geqrs_param(ctx, tree, A, TS, TT, B)
    ref = torch.linalg.lstsq(_dense(A2), b).solution
    assert rel_err(_dense(B)[:30], ref) < 1e-11


def _hqr_worker(rank, world, P, engine="panel"):
    import dplasma_amd as dp
    from dplasma_amd.models import qr_panel
    ctx = dp.init(device="cpu", P=P)
    dt = torch.float64
    A = dp.block_cyclic(ctx, dt, 8, 8, 68, 36)
    dp.plrnt(ctx, A, 3)
    TS = dp.block_cyclic(ctx, dt, 4, 8, A.mt * 4, A.nt * 8)
    TT = dp.block_cyclic(ctx, dt, 4, 8, A.mt * 4, A.nt * 8)
    tree = dp.hqr_init(dp.dplasmaNoTrans, A, dp.dplasma_GREEDY_TREE, dp.dplasma_BINARY_TREE, 2, 2)
    with qr_panel.engine(engine):
        assert qr_panel.usable(A, tree) == (engine == "panel")
        dp.geqrf_param(ctx, tree, A, TS, TT)
        C = dp.block_cyclic(ctx, dt, 8, 8, 68, 10)
        dp.plrnt(ctx, C, 5)
        dp.unmqr_param(ctx, dp.dplasmaLeft, dp.dplasmaConjTrans, tree, A, TS, TT, C)
        D = dp.block_cyclic(ctx, dt, 8, 8, 9, 68)
        dp.plrnt(ctx, D, 6)
        dp.unmqr_param(ctx, dp.dplasmaRight, dp.dplasmaNoTrans, tree, A, TS, TT, D)
    return A.to_dense_local(), TS.to_dense_local(), TT.to_dense_local(), C.to_dense_local(), D.to_dense_local()


@pytest.mark.parametrize("world,P,engine", [(2, 2, "tile"), (4, 2, "tile"), (2, 2, "panel"), (4, 2, "panel"),
                                            (8, 2, "panel")])
def test_hqr_distributed(world, P, engine):
    """geqrf_param + unmqr_param (left and right) on P x Q grids match one process with the same
    engine: the tile DAG, or the stacked-domain engine (process-row TS domains, cross-row TT kills
    exchanging R / V2 / T and the partial W)."""
    out = run_distributed(_hqr_worker, world, P, engine)
    with qr_panel.engine(engine):
        r = _hqr_worker(0, 1, 1, engine)
    for i in range(5):
        assert rel_err(sum(out[k][i] for k in range(world)), r[i]) < 1e-12, i


# one-row trees: every pivot's TT kills of a step are ONE stacked panel of triangles (qr_panel.step_plan)
ONE_ROW_TREES = [(0, 0, 1, 1), (1, 0, 2, 1), (3, 0, 1, 1), (1, 0, -1, 1)]


def test_tt_stack_merge_plan():
    """Merged stacks: each pivot once per step, victims in kill order, never more rounds than the
    pairwise plan, and the greedy chains collapse."""
    ctx_ = dp.init(device="cpu")
    A = dp.block_cyclic(ctx_, torch.float64, 2, 2, 64, 64)
    for ta in ONE_ROW_TREES:
        tree = dp.hqr_init(dp.dplasmaNoTrans, A, *ta)
        n_pair = n_merged = 0
        for k in range(A.nt):
            d1, pairs = qr_panel.step_plan(tree, k, merge=False)
            d2, stacks = qr_panel.step_plan(tree, k, merge=True)
            assert d1 == d2
            assert sorted(m for _, ms in stacks for m in ms) == sorted(ms[0] for _, ms in pairs)
            assert len(stacks) <= 1 and (not pairs or stacks[0][0] == d1[0][0])   # one survivor: the step's head
            n_pair += len(pairs)
            n_merged += len(stacks)
        assert n_merged <= n_pair


@pytest.mark.parametrize("treeargs", [(0, 0, 2, 2), (1, 1, 2, 2), (1, 0, 4, 2), (3, 1, 2, 4), (2, 1, 3, 3)])
def test_tt_row_stack_plan(treeargs):
    """Trees over p process rows (merge="row"): every local stack lies in ONE process row, cross-row kills stay
    pairwise, each victim appears once, the tree's tile pairs are all reduced, and a stack only ever comes
    after the cross-row kills it must follow (its root's and victims' last cross-row use precedes it or none)."""
    ctx_ = dp.init(device="cpu")
    A = dp.block_cyclic(ctx_, torch.float64, 2, 2, 96, 64)
    tree = dp.hqr_init(dp.dplasmaNoTrans, A, *treeargs)
    p = treeargs[3]
    prow = lambda m: m % p  # noqa: E731
    n_pair = n_row = 0
    for k in range(A.nt):
        d1, pairs = qr_panel.step_plan(tree, k, merge=False)
        d2, stacks = qr_panel.step_plan(tree, k, merge="row", prow=prow)
        assert d1 == d2
        assert sorted(m for _, ms in stacks for m in ms) == sorted(ms[0] for _, ms in pairs)
        for (r, ms) in stacks:
            rows = {prow(r)} | {prow(m) for m in ms}
            assert len(rows) == 1 or len(ms) == 1          # cross-row entries are pairs
        dead = set()
        for (r, ms) in stacks:                               # nothing used after it was killed
            assert r not in dead and not (set(ms) & dead)
            dead |= set(ms)
        n_pair += len(pairs)
        n_row += len(stacks)
    assert n_row <= n_pair


@pytest.mark.parametrize("prec", list("dz"))
@pytest.mark.parametrize("treeargs", ONE_ROW_TREES)
def test_hqr_one_row_tree(ctx, prec, treeargs):
    M, N = 70, 40
    e1, e2, *_ = _hqr_run(ctx, DTYPES[prec], False, treeargs, M, N, 8, 4)
    assert e1 < 1e-13 and e2 < 1e-13


@pytest.mark.parametrize("knobs", [{"DPLASMA_QR_MERGE_TT": "0"}, {"DPLASMA_QR_VT": "0"},
                                   {"DPLASMA_QR_LOOKAHEAD": "0"}, {"DPLASMA_QR_BATCHED": "0"}])
def test_hqr_engine_knobs(ctx, monkeypatch, knobs):
    """The stacked-domain engine's alternatives (pairwise TT kills, T applied to W, no look-ahead, entry by
    entry) factor the same matrix as the default path (same R up to row signs, orthogonal Q)."""
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    for ta in ONE_ROW_TREES[:2]:
        e1, e2, A, *_ = _hqr_run(ctx, torch.float64, False, ta, 70, 40, 8, 4)
        assert e1 < 1e-13 and e2 < 1e-13
        monkeypatch.delenv(next(iter(knobs)))
        _, _, B, *_ = _hqr_run(ctx, torch.float64, False, ta, 70, 40, 8, 4)
        monkeypatch.setenv(*next(iter(knobs.items())))
        ra, rb = torch.triu(_dense(A)[:40]).abs(), torch.triu(_dense(B)[:40]).abs()
        assert rel_err(ra, rb) < 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("prec", list("ds"))
@pytest.mark.parametrize("treeargs", ONE_ROW_TREES)
def test_gpu_hqr_one_row_tree(gctx, ctx, prec, treeargs):
    """Merged TT stacks through the GPU panel kernel vs the same plan on the CPU."""
    dt = DTYPES[prec]
    res = [_hqr_run(c, dt, False, treeargs, 600, 320, 32, 8) for c in (gctx, ctx)]
    lim = 1e-4 if prec == "s" else 1e-12
    assert res[0][0] < lim and res[0][1] < lim
    assert rel_err(_dense(res[0][2]), _dense(res[1][2])) < lim * 10


@pytest.mark.gpu
@pytest.mark.parametrize("prec", list("sdcz"))
@pytest.mark.parametrize("lq", [False, True])
def test_gpu_hqr(gctx, ctx, prec, lq):
    dt = DTYPES[prec]
    M, N = (300, 160) if not lq else (160, 300)
    res = [_hqr_run(c, dt, lq, (1, 3, 2, 2), M, N, 32, 8) for c in (gctx, ctx)]
    lim = 1e-4 if prec in "sc" else 1e-12
    assert res[0][0] < lim and res[0][1] < lim
    assert rel_err(_dense(res[0][2]), _dense(res[1][2])) < lim * 10


# ----------------------------------------------------------------------------- stacked-domain engine
def _panel_case(device, dt, M, nc, kf, ld, seed):
    from dplasma_amd.ops import tile_ops as ops
    g = torch.Generator().manual_seed(seed)
    Pc = torch.randn(M, nc, generator=g, dtype=torch.float64)
    P = torch.zeros(ld * nc, dtype=dt, device=device)
    torch.as_strided(P, (M, nc), (1, ld), 0).copy_(Pc.to(dt))
    V = torch.zeros(ld * kf, dtype=dt, device=device)
    Tm = torch.zeros(kf * kf, dtype=dt, device=device)
    ws = ops.qr_panel_workspace(nc, kf, dt, device)
    info = torch.zeros(1, dtype=torch.int32, device=device)
    ops.qr_panel(P, ld, M, nc, kf, V, ld, Tm, kf, ws, info)
    out = (torch.as_strided(P, (M, nc), (1, ld), 0).cpu().double(), torch.as_strided(V, (M, kf), (1, ld), 0).cpu().double(),
           torch.as_strided(Tm, (kf, kf), (1, kf), 0).cpu().double())
    return Pc, out, int(info.item())


@pytest.mark.parametrize("M,nc,kf", [(40, 16, 16), (23, 30, 23), (70, 40, 40)])
def test_qr_panel_op_cpu(M, nc, kf):
    """The panel op's CPU path: Q = I - V T V^T is orthogonal and Q^T P0 = [R; 0] (+ updated columns)."""
    P0, (P, V, T), _ = _panel_case("cpu", torch.float64, M, nc, kf, M + 5, 1)
    Q = torch.eye(M, dtype=torch.float64) - V @ T @ V.T
    assert (Q.T @ Q - torch.eye(M, dtype=torch.float64)).abs().max() < 1e-13
    R = torch.triu(P[:, :kf])
    ref = Q.T @ P0
    assert rel_err(torch.triu(ref[:, :kf]), R) < 1e-13
    if M > kf:
        assert ref[kf:, :kf].abs().max() < 1e-12
    if nc > kf:
        assert rel_err(ref[:, kf:], P[:, kf:]) < 1e-13


@pytest.mark.parametrize("M,N,NB,IB,tree,st", [(96, 64, 16, 4, None, "tile"), (90, 90, 16, 8, None, "tile"),
                                               (100, 48, 16, 4, (1, 1, 2, 1), "tile"), (100, 48, 16, 4, (0, 3, 3, 1), "tile"),
                                               (64, 96, 16, 4, None, "tile"), (90, 70, 16, 4, None, "lapack")])
def test_qr_panel_engine_cpu(ctx, M, N, NB, IB, tree, st):
    """geqrf / geqrf_param through the stacked-domain engine: factors, Q and its applications."""
    dt = torch.float64
    A = _mk(ctx, dt, M, N, NB, 5, storage=st)
    a = _dense(A)
    TS, TT = _T(ctx, A, IB), _T(ctx, A, IB)
    tr = dp.hqr_init(dp.dplasmaNoTrans, A, *tree) if tree else None
    assert qr_panel.usable(A, tr or dp.models.qrtree.FlatTree(A.mt, A.nt))
    if tr is None:
        dp.geqrf(ctx, A, TS)
    else:
        dp.geqrf_param(ctx, tr, A, TS, TT)
    K = min(M, N)
    Q = dp.block_cyclic(ctx, dt, NB, NB, M, M)
    if tr is None:
        dp.ungqr(ctx, A, TS, Q)
    else:
        dp.ungqr_param(ctx, tr, A, TS, TT, Q)
    q = _dense(Q)
    assert (q.T @ q - torch.eye(M, dtype=dt)).abs().max() < 1e-13
    assert rel_err(q[:, :K] @ torch.triu(_dense(A)[:K]), a) < 1e-13
    for side in (dp.dplasmaLeft, dp.dplasmaRight):
        for trans in (dp.dplasmaNoTrans, dp.dplasmaTrans):
            shp = (M, 11) if side == dp.dplasmaLeft else (11, M)
            C = _mk(ctx, dt, shp[0], shp[1], NB, 9)
            c = _dense(C)
            if tr is None:
                dp.unmqr(ctx, side, trans, A, TS, C)
            else:
                dp.unmqr_param(ctx, side, trans, tr, A, TS, TT, C)
            op = q if trans == dp.dplasmaNoTrans else q.T
            ref = op @ c if side == dp.dplasmaLeft else c @ op
            assert rel_err(_dense(C), ref) < 1e-12, (side, trans)


@pytest.mark.gpu
@pytest.mark.parametrize("prec", ["d", "s"])
@pytest.mark.parametrize("M,nc,kf", [(300, 64, 64), (1000, 256, 256), (256, 256, 256), (513, 200, 200), (70, 100, 70),
                                     (5000, 256, 256), (40000, 256, 256), (65536, 128, 128)])
def test_gpu_qr_panel_kernel(prec, M, nc, kf):
    """Persistent HIP panel kernel vs the LAPACK path of the same op (same sign conventions)."""
    dt = DTYPES[prec]
    ld = M + 7
    P0, g, info = _panel_case("cuda", dt, M, nc, kf, ld, M + nc)
    assert info == 0
    _, c, _ = _panel_case("cpu", torch.float64, M, nc, kf, ld, M + nc)
    tol = 1e-10 if prec == "d" else 2e-3
    for i, (x, y) in enumerate(zip(g, c)):
        assert rel_err(x, y) < tol, i


@pytest.mark.gpu
@pytest.mark.parametrize("M,nc", [(700, 96), (256, 256), (3000, 128)])
def test_gpu_qr_panel_kernel_rank_deficient(M, nc):
    """Columns that make the kernel's Gram-downdated norms cancel (exact copies, 1e-10
    perturbations, zero columns, the last rows of a square panel) take the exact reduction path:
    Q = I - V T V^T stays orthogonal and Q^T P0 = [R; 0] to working precision."""
    from dplasma_amd.ops import tile_ops as ops
    dev, dt = "cuda", torch.float64
    g = torch.Generator().manual_seed(7)
    P0 = torch.randn(M, nc, generator=g, dtype=dt)
    P0[:, 5] = P0[:, 3]
    P0[:, 9] = P0[:, 2] + 1e-10 * torch.randn(M, generator=g, dtype=dt)
    P0[:, 40] = 0.0
    P0[:, 41] = 1e-3 * P0[:, 0] - 2.0 * P0[:, 33]
    ld = M + 3
    P = torch.zeros(ld * nc, dtype=dt, device=dev)
    torch.as_strided(P, (M, nc), (1, ld), 0).copy_(P0.to(dev))
    V = torch.zeros(ld * nc, dtype=dt, device=dev)
    Tm = torch.zeros(nc * nc, dtype=dt, device=dev)
    ws = ops.qr_panel_workspace(nc, nc, dt, dev)
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    ops.qr_panel(P, ld, M, nc, nc, V, ld, Tm, nc, ws, info)
    assert int(info.item()) == 0
    Pf = torch.as_strided(P, (M, nc), (1, ld), 0).cpu()
    Vf = torch.as_strided(V, (M, nc), (1, ld), 0).cpu()
    Tf = torch.as_strided(Tm, (nc, nc), (1, nc), 0).cpu()
    Q = torch.eye(M, dtype=dt) - Vf @ Tf @ Vf.T
    assert (Q.T @ Q - torch.eye(M, dtype=dt)).abs().max() < 1e-13
    ref = Q.T @ P0
    assert rel_err(torch.triu(ref[:nc]), torch.triu(Pf[:nc])) < 1e-13
    if M > nc:
        assert ref[nc:].abs().max() < 1e-12 * P0.abs().max()


def _qrp_worker(rank, world, P):
    """Stacked-domain engine on a 1 x Q grid (flat and one-domain HQR trees)."""
    import dplasma_amd as dp
    ctx = dp.init(device="cpu", P=P)
    dt = torch.float64
    M, N, NB, IB = 72, 56, 8, 4
    out = []
    for use_tree in (False, True):
        A = dp.block_cyclic(ctx, dt, NB, NB, M, N)
        dp.plrnt(ctx, A, 3872)
        TS = dp.block_cyclic(ctx, dt, IB, NB, A.mt * IB, A.nt * NB)
        TT = dp.block_cyclic(ctx, dt, IB, NB, A.mt * IB, A.nt * NB)
        tree = dp.hqr_init(dp.dplasmaNoTrans, A, 1, 1, A.mt, 1) if use_tree else None
        assert qr_panel.usable(A, tree or dp.models.qrtree.FlatTree(A.mt, A.nt))
        if use_tree:
            dp.geqrf_param(ctx, tree, A, TS, TT)
        else:
            dp.geqrf(ctx, A, TS)
        Q = dp.block_cyclic(ctx, dt, NB, NB, M, M)
        C1 = dp.block_cyclic(ctx, dt, NB, NB, M, 20)
        C2 = dp.block_cyclic(ctx, dt, NB, NB, 12, M)
        dp.plrnt(ctx, C1, 5)
        dp.plrnt(ctx, C2, 6)
        if use_tree:
            dp.ungqr_param(ctx, tree, A, TS, TT, Q)
            dp.unmqr_param(ctx, dp.dplasmaLeft, dp.dplasmaTrans, tree, A, TS, TT, C1)
            dp.unmqr_param(ctx, dp.dplasmaRight, dp.dplasmaNoTrans, tree, A, TS, TT, C2)
        else:
            dp.ungqr(ctx, A, TS, Q)
            dp.unmqr(ctx, dp.dplasmaLeft, dp.dplasmaTrans, A, TS, C1)
            dp.unmqr(ctx, dp.dplasmaRight, dp.dplasmaNoTrans, A, TS, C2)
        out += [A.to_dense_local(), TS.to_dense_local(), Q.to_dense_local(), C1.to_dense_local(),
                C2.to_dense_local()]
    return out


@pytest.mark.parametrize("world", [2, 3])
def test_qr_panel_engine_1xq(world):
    out = run_distributed(_qrp_worker, world, 1)
    r = _qrp_worker(0, 1, 1)
    for i in range(len(r)):
        full = sum(out[k][i] for k in range(world))
        assert rel_err(full, r[i]) < 1e-12, i


@pytest.mark.parametrize("mt,nt,flat,greedy", [(1, 1, 4, 4), (2, 1, 10, 6), (2, 2, 26, 20), (4, 4, 86, 64),
                                               (16, 2, 196, 48)])
def test_qr_simulation_date(mt, nt, flat, greedy):
    """Critical path of the tile QR DAG with the reference SIMCOST weights (geqrt 4, unmqr 6,
    tsqrt 6 / ttqrt 2, tsmqr 12 / ttmqr 6).  Small cases by hand: 2x1 flat = geqrt + tsqrt = 10,
    greedy = max(geqrt, geqrt) + ttqrt = 6; 2x2 flat = geqrt, then unmqr || tsqrt, tsmqr, geqrt = 26."""
    from dplasma_amd.models import qr_panel
    ctx = dp.init(device="cpu")
    NB, ib = 16, 4
    A = dp.block_cyclic(ctx, torch.float64, NB, NB, mt * NB, nt * NB)
    TS = dp.block_cyclic(ctx, torch.float64, ib, NB, mt * ib, nt * NB)
    TT = TS.like()
    with qr_panel.engine("tile"):
        assert dp.geqrf_New(ctx, A, TS).simulation_date() == flat
        # the reference's fibonacci low-level tree (DPLASMA_FIBONACCI_TREE = 2, dplasma_hqr.c:507-543)
        tree = dp.hqr_init(dp.dplasmaNoTrans, A, 2, 0, 1, 1, False, False)
        assert dp.geqrf_param_New(ctx, tree, A, TS, TT).simulation_date() == greedy
        # the systolic tree with one domain reduces to the flat TS tree
        assert dp.geqrf_param_New(ctx, dp.systolic_init(dp.dplasmaNoTrans, A, 1, 1), A, TS, TT) \
            .simulation_date() == flat
        # unit costs: the date is the DAG depth
        assert dp.geqrf_New(ctx, A, TS).simulation_date(lambda name: 1) >= mt + nt - 1


def _kept_vs_rebuilt(c, dt):
    """ungqr with the T kept by the stacked-domain factorisation vs with T rebuilt from the stored
    diagonal blocks and V (MFMA GEMM engine on the GPU): same Q."""
    M, N, NB, IB = 300, 200, 64, 16
    with qr_panel.engine("panel"):
        A = dp.block_cyclic(c, dt, NB, NB, M, N)
        dp.plrnt(c, A, 3872)
        T = dp.block_cyclic(c, dt, IB, NB, A.mt * IB, A.nt * NB)
        dp.geqrf(c, A, T)
        assert getattr(T, "full_T", None)
        Q1 = dp.block_cyclic(c, dt, NB, NB, M, N)
        dp.ungqr(c, A, T, Q1)
        T.full_T = {}
        Q2 = dp.block_cyclic(c, dt, NB, NB, M, N)
        dp.ungqr(c, A, T, Q2)
    return rel_err(_dense(Q2), _dense(Q1))


@pytest.mark.parametrize("prec", ["d", "s"])   # the stacked-domain engine is real-precision only
def test_qr_kept_T_matches_rebuilt(ctx, prec):
    assert _kept_vs_rebuilt(ctx, DTYPES[prec]) < (1e-4 if prec == "s" else 1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("prec", ["d", "s"])
def test_gpu_qr_kept_T_matches_rebuilt(gctx, prec):
    assert _kept_vs_rebuilt(gctx, DTYPES[prec]) < (1e-4 if prec == "s" else 1e-11)


def _hqr_check_worker(rank, world, P, treeargs, M, N, NB, IB):
    import dplasma_amd as dp
    from dplasma_amd.models import qr_panel
    ctx = dp.init(device="cpu", P=P)
    dt = torch.float64
    A = dp.block_cyclic(ctx, dt, NB, NB, M, N)
    dp.plrnt(ctx, A, 3872)
    TS = dp.block_cyclic(ctx, dt, IB, NB, A.mt * IB, A.nt * NB)
    TT = dp.block_cyclic(ctx, dt, IB, NB, A.mt * IB, A.nt * NB)
    tree = dp.hqr_init(dp.dplasmaNoTrans, A, *treeargs)
    used = qr_panel.usable(A, tree)
    dp.geqrf_param(ctx, tree, A, TS, TT)
    K = min(M, N)
    Q = dp.block_cyclic(ctx, dt, NB, NB, M, K)
    dp.ungqr_param(ctx, tree, A, TS, TT, Q)
    B = dp.block_cyclic(ctx, dt, NB, NB, M, 3)
    dp.plrnt(ctx, B, 11)
    dp.geqrs_param(ctx, tree, A, TS, TT, B)
    return used, A.to_dense_local(), Q.to_dense_local(), B.to_dense_local()


@pytest.mark.parametrize("world,P,treeargs", [(4, 2, (0, 0, 3, 2)), (4, 2, (1, 3, 2, 2)), (8, 2, (1, 0, 4, 2)),
                                              (8, 4, (3, 1, 2, 4))])
def test_hqr_engine_distributed_checks(world, P, treeargs):
    """The reference's testing_zgeqrf_hqr checks on P x Q grids with the stacked-domain engine:
    ||I - Q^T Q||, ||A - Q R|| / ||A|| and the least-squares solve, from the distributed factors."""
    M, N, NB, IB = 96, 56, 8, 4
    out = run_distributed(_hqr_check_worker, world, P, treeargs, M, N, NB, IB)
    assert all(out[r][0] for r in range(world))   # the distributed engine ran
    R = torch.triu(sum(out[r][1] for r in range(world))[:N])
    Qd = sum(out[r][2] for r in range(world))
    X = sum(out[r][3] for r in range(world))[:N]
    ctx = dp.Context(device="cpu")
    A0 = _mk(ctx, torch.float64, M, N, NB, 3872).to_dense_local()
    B0 = _mk(ctx, torch.float64, M, 3, NB, 11).to_dense_local()
    assert (Qd.T @ Qd - torch.eye(N, dtype=torch.float64)).abs().max() < 1e-13
    assert (Qd @ R - A0).abs().max() / A0.abs().max() < 1e-13
    assert rel_err(X, torch.linalg.lstsq(A0, B0).solution) < 1e-11
