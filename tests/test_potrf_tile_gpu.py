"""Diagonal-tile Cholesky kernels on the GPU against a plain PyTorch fp64 reference.

Covers the multi-workgroup dataflow kernel (csrc/kernels/potrf_rb.hip, fp64 n <= 512) and the
single-workgroup kernel it replaces (potrf_trsm.hip), both through ``ops.potrf_tile``:
odd sizes (identity padding of the last 32-row block), lower/upper storage, a leading dimension
larger than n, the untouched opposite triangle, LAPACK's info convention on a non-SPD tile, and
repeated launches while a large GEMM keeps every CU busy on another stream (the workgroup
hand-offs must hold under uneven load).
"""
import pytest
import torch

from dplasma_amd.constants import dplasmaLower, dplasmaUpper

pytestmark = pytest.mark.gpu


def _lib():
    from dplasma_amd.ops import _lib
    return _lib.load()


def _spd(n, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    M = torch.randn(n, n, dtype=torch.float64, generator=g)
    return (M @ M.T + n * torch.eye(n, dtype=torch.float64)).cuda()


def _run(kind, uplo, S, lda, info_base=0):
    from dplasma_amd.ops import tile_ops as ops
    n = S.shape[0]
    buf = torch.full((lda * n,), 7.0, dtype=torch.float64, device="cuda")
    view = torch.as_strided(buf, (n, n), (1, lda), 0)
    view.copy_(S)
    info = torch.zeros(1, dtype=torch.int32, device="cuda")
    old = _lib().dpl_potrf_tile_set_kind(kind)
    try:
        ops.potrf_tile(uplo, buf, 0, n, lda, info, info_base)
        torch.cuda.synchronize()
    finally:
        _lib().dpl_potrf_tile_set_kind(old)
    return view.clone(), int(info.item()), buf


@pytest.mark.parametrize("kind", [0, 1])
@pytest.mark.parametrize("uplo", [dplasmaLower, dplasmaUpper])
@pytest.mark.parametrize("n", [1, 31, 32, 33, 100, 256, 480, 511, 512])
def test_potrf_tile_vs_torch(kind, uplo, n):
    S = _spd(n, seed=n)
    lda = n + 9
    out, info, _ = _run(kind, uplo, S, lda)
    assert info == 0
    Lref = torch.linalg.cholesky(S)
    if uplo == dplasmaLower:
        got, other, ref_other = out.tril(), out.triu(1), S.triu(1)
        ref = Lref
    else:
        got, other, ref_other = out.triu(), out.tril(-1), S.tril(-1)
        ref = Lref.T
    err = (got - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-13, err
    # the opposite strict triangle is never written
    assert torch.equal(other, ref_other)


@pytest.mark.parametrize("kind", [0, 1])
@pytest.mark.parametrize("bad", [0, 5, 31, 32, 200, 511])
def test_potrf_tile_info(kind, bad):
    n = 512
    S = _spd(n, seed=3)
    # make the leading minor of order bad+1 indefinite: the first failing column is `bad`
    L = torch.linalg.cholesky(S)
    S = S.clone()
    S[bad, bad] -= 2 * (L[bad, bad] ** 2)
    _, info, _ = _run(kind, dplasmaLower, S, n, info_base=1000)
    assert info == 1000 + bad + 1


def test_potrf_tile_under_load():
    """Repeated dataflow-kernel launches on a high-priority stream while a big MFMA GEMM occupies
    every CU on another stream: every factorisation must be exact."""
    from dplasma_amd.ops import tile_ops as ops
    from dplasma_amd.ops.batch import GemmBatch
    n, lda = 512, 512
    S = _spd(n, seed=11)
    Lref = torch.linalg.cholesky(S)
    N = 8192
    big = torch.randn(3 * N * N, dtype=torch.float64, device="cuda")
    gb = GemmBatch()
    for i in range(0, N, 512):
        for j in range(0, N, 512):
            gb.add(2 * N * N + i + j * N, 512, 512, [(i, N * N + j * N, N)], 0)
    gb.finalize()
    lo = torch.cuda.Stream(priority=0)
    hi = torch.cuda.Stream(priority=-1)
    reps = 24
    bufs = [torch.empty(n * lda, dtype=torch.float64, device="cuda") for _ in range(reps)]
    infos = torch.zeros(reps, dtype=torch.int32, device="cuda")
    for b in bufs:
        torch.as_strided(b, (n, n), (1, lda), 0).copy_(S)
    torch.cuda.synchronize()
    with torch.cuda.stream(lo):
        from dplasma_amd.constants import dplasmaNoTrans
        ops.gemm(dplasmaNoTrans, dplasmaNoTrans, 1.0, big, N, big, N, 0.0, big, N, gb)
    with torch.cuda.stream(hi):
        for r in range(reps):
            ops.potrf_tile(dplasmaLower, bufs[r], 0, n, lda, infos[r:r + 1], 0)
    torch.cuda.synchronize()
    assert int(infos.abs().max().item()) == 0
    for b in bufs:
        got = torch.as_strided(b, (n, n), (1, lda), 0).tril()
        assert (got - Lref).abs().max().item() < 1e-12


@pytest.mark.parametrize("uplo", [dplasmaLower, dplasmaUpper])
@pytest.mark.parametrize("n", [512, 100, 32])
@pytest.mark.parametrize("prep", [False, True, "fused"])
def test_trsm_rb_panel(uplo, n, prep):
    """Panel solve of the Cholesky step (k_trsm_rb) against torch.linalg.solve_triangular, with the
    inverted diagonal blocks from the tile factorisation itself or from k_trsm_rb_prep."""
    from dplasma_amd.ops import tile_ops as ops
    S = _spd(n, seed=7 + n)
    ms = [n, 77, n, 1]
    ld = n + sum(ms) + 5
    g = torch.Generator(device="cpu").manual_seed(n)
    Bs = [torch.randn(m, n, dtype=torch.float64, generator=g).cuda() for m in ms]  # lower view: m x n
    # storage: tile 0 = diagonal, then the panel tiles (lower: below it; upper: to its right)
    buf = torch.zeros(ld * (n * 5 + 100), dtype=torch.float64, device="cuda")
    def view(off, r, c):
        return torch.as_strided(buf, (r, c), (1, ld), off)
    view(0, n, n).copy_(S)
    offs, tiles = [], []
    if uplo == dplasmaLower:
        r0 = n
        for B, m in zip(Bs, ms):
            view(r0, m, n).copy_(B)
            offs.append(r0); tiles.append((r0, m)); r0 += m
    else:
        c0 = n
        for B, m in zip(Bs, ms):
            view(c0 * ld, n, m).copy_(B.T)
            offs.append(c0 * ld); tiles.append((c0 * ld, m)); c0 += m
    info = torch.zeros(1, dtype=torch.int32, device="cuda")
    zbuf = torch.zeros(ops.rb_zbuf_size(), dtype=torch.float64, device="cuda")
    panel = ops.RbPanel(uplo, tiles, ld)
    if prep == "fused":   # one launch: tile factorisation + panel strips along its wavefront
        ops.potrf_trsm_rb(uplo, n, buf, 0, ld, info, 0, zbuf, panel, buf, ld)
    else:
        ops.potrf_tile(uplo, buf, 0, n, ld, info, 0, zbuf=zbuf)
        if prep:
            zbuf.fill_(float("nan"))
            ops.trsm_rb_prep(uplo, n, buf, 0, ld, zbuf)
        ops.trsm_rb(uplo, n, buf, 0, ld, zbuf, panel, buf, ld)
    torch.cuda.synchronize()
    assert int(info.item()) == 0
    L = torch.linalg.cholesky(S)
    tri = view(0, n, n).tril() if uplo == dplasmaLower else view(0, n, n).triu().T
    assert (tri - L).abs().max().item() < 1e-12 * max(1.0, L.abs().max().item())
    for B, m, off in zip(Bs, ms, offs):
        ref = torch.linalg.solve_triangular(L, B.T, upper=False).T  # B L^{-T}
        got = view(off, m, n) if uplo == dplasmaLower else view(off, n, m).T
        err = (got - ref).abs().max().item() / max(1.0, ref.abs().max().item())
        assert err < 1e-12, (m, err)


@pytest.mark.parametrize("uplo", [dplasmaLower, dplasmaUpper])
@pytest.mark.parametrize("N,NB", [(4096, 512), (3000, 384), (2048, 256)])
def test_potrf_fused_trsm(uplo, N, NB, monkeypatch):
    """Whole DPOTRF with the fused tile + panel-solve launch (DPLASMA_POTRF_TRSM=fused) passes the
    reference check (src/dplasma_zcheck.c check_zpotrf) and matches the default two-launch path."""
    import dplasma_amd as dp
    ctx = dp.init(device="cuda:0")
    out = {}
    for kind in ("rb", "fused"):
        monkeypatch.setenv("DPLASMA_POTRF_TRSM", kind)
        A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
        dp.dplghe(ctx, float(N), uplo, A, 3872)
        A0 = A.like()
        dp.lacpy(ctx, dp.dplasmaUpperLower, A, A0)
        assert dp.dpotrf(ctx, uplo, A) == 0
        ok, res = dp.check_potrf(ctx, uplo, A, A0)
        assert ok, (kind, res)
        out[kind] = A.to_dense_local()
    tri = (lambda x: x.tril()) if uplo == dplasmaLower else (lambda x: x.triu())
    assert (tri(out["rb"]) - tri(out["fused"])).abs().max().item() < 1e-10
