"""ScaLAPACK shims on caller-owned block-cyclic local arrays (zero-copy LAPACK-storage descriptors)."""
import pytest
import torch

from helpers import rel_err, run_distributed


def _to_local(G, mb, nb, P, Q, myrow, mycol, rsrc=0, csrc=0):
    """Global dense -> ScaLAPACK local array (column-major, lld = local rows), flat."""
    from dplasma_amd.scalapack import numroc
    m, n = G.shape
    lr = numroc(m, mb, myrow, rsrc, P)
    lc = numroc(n, nb, mycol, csrc, Q)
    L = torch.zeros(max(lr, 1), max(lc, 1), dtype=G.dtype)
    rows = [i for i in range(m) if ((i // mb + P - rsrc) % P) == myrow]
    cols = [j for j in range(n) if ((j // nb + Q - csrc) % Q) == mycol]
    if rows and cols:
        L[:len(rows), :len(cols)] = G[rows][:, cols]
    return L.t().contiguous().reshape(-1), max(lr, 1), rows, cols


def _from_local(flat, lld, rows, cols, m, n, dtype):
    G = torch.zeros(m, n, dtype=dtype)
    if rows and cols:
        L = flat.reshape(-1, lld).t()
        G[torch.tensor(rows)[:, None], torch.tensor(cols)[None, :]] = L[:len(rows), :len(cols)]
    return G


def _worker(rank, world, P):
    import dplasma_amd as dp
    from dplasma_amd import scalapack as sl
    ctx = dp.init(device="cpu", P=P)
    Q = world // P
    myrow, mycol = rank // Q, rank % Q
    ictxt = sl.blacs_gridinit(ctx)
    g = torch.Generator().manual_seed(7)
    n, mb = 45, 8
    out = {}
    # pdpotrf_
    X = torch.randn(n, n, generator=g, dtype=torch.float64)
    S = X @ X.T + n * torch.eye(n, dtype=torch.float64)
    a, lld, rows, cols = _to_local(S, mb, mb, P, Q, myrow, mycol)
    desc = sl.descinit(n, n, mb, mb, 0, 0, ictxt, lld)
    out["potrf_info"] = sl.pdpotrf_("L", n, a, 1, 1, desc)
    out["potrf"] = _from_local(a, lld, rows, cols, n, n, torch.float64)
    # pdgemm_ (sub-matrix, tile aligned)
    A = torch.randn(n, n, generator=g, dtype=torch.float64)
    B = torch.randn(n, n, generator=g, dtype=torch.float64)
    C = torch.randn(n, n, generator=g, dtype=torch.float64)
    la, lda, ra, ca = _to_local(A, mb, mb, P, Q, myrow, mycol)
    lb, ldb, rb, cb = _to_local(B, mb, mb, P, Q, myrow, mycol)
    lc, ldc, rc, cc = _to_local(C, mb, mb, P, Q, myrow, mycol)
    sl.pdgemm_("N", "T", n - 8, n - 8, n - 16, 2.0, la, 9, 17, sl.descinit(n, n, mb, mb, 0, 0, ictxt, lda),
               lb, 9, 17, sl.descinit(n, n, mb, mb, 0, 0, ictxt, ldb), 0.5, lc, 9, 9,
               sl.descinit(n, n, mb, mb, 0, 0, ictxt, ldc))
    out["gemm"] = (_from_local(lc, ldc, rc, cc, n, n, torch.float64), A, B, C)
    # pdgetrf_ + ipiv
    la, lda, ra, ca = _to_local(A, mb, mb, P, Q, myrow, mycol)
    ipiv = torch.zeros(lda + mb, dtype=torch.int32)
    out["getrf_info"] = sl.pdgetrf_(n, n, la, 1, 1, sl.descinit(n, n, mb, mb, 0, 0, ictxt, lda), ipiv)
    out["getrf"] = _from_local(la, lda, ra, ca, n, n, torch.float64)
    out["ipiv"] = {r: int(ipiv[i]) for i, r in enumerate(ra)}
    # pdtrsm_ / pdtrmm_
    T = torch.triu(torch.randn(n, n, generator=g, dtype=torch.float64)) + n * torch.eye(n, dtype=torch.float64)
    lt, ldt, rt, ct_ = _to_local(T, mb, mb, P, Q, myrow, mycol)
    lb, ldb, rb, cb = _to_local(B, mb, mb, P, Q, myrow, mycol)
    sl.pdtrsm_("L", "U", "N", "N", n, n, 1.0, lt, 1, 1, sl.descinit(n, n, mb, mb, 0, 0, ictxt, ldt),
               lb, 1, 1, sl.descinit(n, n, mb, mb, 0, 0, ictxt, ldb))
    out["trsm"] = (_from_local(lb, ldb, rb, cb, n, n, torch.float64), T, B)
    sl.pdtrmm_("L", "U", "N", "N", n, n, 1.0, lt, 1, 1, sl.descinit(n, n, mb, mb, 0, 0, ictxt, ldt),
               lb, 1, 1, sl.descinit(n, n, mb, mb, 0, 0, ictxt, ldb))
    out["trmm"] = _from_local(lb, ldb, rb, cb, n, n, torch.float64)
    # pdlatsqr_ (tall skinny)
    m2, n2 = 80, 16
    W = torch.randn(m2, n2, generator=g, dtype=torch.float64)
    lw, ldw, rw, cw = _to_local(W, mb, mb, P, Q, myrow, mycol)
    info, TS, TT, tree = sl.pdlatsqr_(m2, n2, lw, 1, 1, sl.descinit(m2, n2, mb, mb, 0, 0, ictxt, ldw))
    out["latsqr"] = (_from_local(lw, ldw, rw, cw, m2, n2, torch.float64), W)
    return _np(out)


def _np(x):
    """Plain numpy payloads: tensors sent through the mp queue would live in the worker's shared memory."""
    if isinstance(x, torch.Tensor):
        return x.numpy().copy()
    if isinstance(x, dict):
        return {k: _np(v) for k, v in x.items()}
    if isinstance(x, tuple):
        return tuple(_np(v) for v in x)
    return x


def _t(x):
    if isinstance(x, dict):
        return {k: _t(v) for k, v in x.items()}
    if isinstance(x, tuple):
        return tuple(_t(v) for v in x)
    import numpy as np
    return torch.from_numpy(x) if isinstance(x, np.ndarray) else x


@pytest.mark.parametrize("world,P", [(1, 1), (4, 2), (2, 2)])
def test_scalapack_shims(world, P):
    if world == 1:
        outs = {0: _worker(0, 1, 1)}
    else:
        outs = run_distributed(_worker, world, P)
    outs = {r: _t(v) for r, v in outs.items()}
    tot = lambda key, i=None: sum((outs[r][key] if i is None else outs[r][key][i]) for r in range(world))  # noqa
    S = None
    r0 = outs[0]
    # potrf
    assert all(outs[r]["potrf_info"] == 0 for r in range(world))
    Lf = torch.tril(tot("potrf"))
    A, B, C = r0["gemm"][1:]
    # gemm: rows/cols 8: of C updated with op(A(8:, 16:)) op(B(8:,16:))^T
    Cg = tot("gemm", 0)
    ref = C.clone()
    ref[8:, 8:] = 2.0 * A[8:, 16:] @ B[8:, 16:].T + 0.5 * C[8:, 8:]
    assert rel_err(Cg, ref) < 1e-12
    # getrf
    lu, piv = torch.linalg.lu_factor(A)
    assert rel_err(tot("getrf"), lu) < 1e-12
    ip = {}
    for r in range(world):
        ip.update(outs[r]["ipiv"])
    assert all(ip[i] == int(piv[i]) for i in range(A.shape[0]))
    # trsm then trmm gives B back
    T = r0["trsm"][1]
    assert rel_err(tot("trsm", 0), torch.linalg.solve_triangular(T, B, upper=True)) < 1e-12
    assert rel_err(tot("trmm"), B) < 1e-12
    # latsqr: |R| matches the R of LAPACK QR up to signs
    R = torch.triu(tot("latsqr", 0)[:16])
    W = r0["latsqr"][1]
    Rref = torch.linalg.qr(W).R
    assert rel_err(R.abs(), Rref.abs()) < 1e-10
