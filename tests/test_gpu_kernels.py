"""GPU numerics: every HIP kernel vs the CPU/PyTorch fp64 reference of the same op."""
import pytest
import torch

import dplasma_amd as dp
from dplasma_amd.ops import _lib
from dplasma_amd.ops import tile_ops as ops
from dplasma_amd.ops.batch import TileBatch
from helpers import DTYPES, rel_err, tol

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gctx():
    _lib.load()
    return dp.init(device="cuda:0")


@pytest.fixture(scope="module")
def cctx():
    return dp.Context(device="cpu")


def test_native_library_loaded(gctx):
    maps = open("/proc/self/maps").read()
    assert "libdplasma_kernels.so" in maps


def _pair(gctx, cctx, dt, mb, nb, m, n, storage=dp.STORAGE_TILE):
    G = dp.block_cyclic(gctx, dt, mb, nb, m, n, storage=storage)
    C = dp.block_cyclic(cctx, dt, mb, nb, m, n, storage=storage)
    return G, C


@pytest.mark.parametrize("prec", list("sdcz"))
@pytest.mark.parametrize("kind", ["rnt", "ghe", "gsy"])
def test_generators_bit_identical(gctx, cctx, prec, kind):
    dt = DTYPES[prec]
    G, C = _pair(gctx, cctx, dt, 37, 37, 150, 150)
    for ctx, X in ((gctx, G), (cctx, C)):
        if kind == "rnt":
            dp.plrnt(ctx, X, 3872)
        elif kind == "ghe":
            dp.plghe(ctx, 150.0, dp.dplasmaUpperLower, X, 3872)
        else:
            dp.plgsy(ctx, 150.0, dp.dplasmaUpperLower, X, 3872)
    torch.cuda.synchronize()
    assert torch.equal(G.to_dense_local(), C.to_dense_local())


@pytest.mark.parametrize("prec", list("sdcz"))
@pytest.mark.parametrize("ta,tb", [(111, 111), (111, 112), (112, 111), (112, 112), (113, 111), (111, 113)])
@pytest.mark.parametrize("dims", [(300, 280, 256, 128), (106, 283, 97, 56), (512, 512, 512, 512)])
def test_gemm(gctx, cctx, prec, ta, tb, dims):
    if prec in "sd" and (ta == 113 or tb == 113):
        pytest.skip("conj == trans for real")
    dt = DTYPES[prec]
    M, N, K, NB = dims
    am, an = (M, K) if ta == 111 else (K, M)
    bm, bn = (K, N) if tb == 111 else (N, K)
    res = []
    for ctx in (gctx, cctx):
        A = dp.block_cyclic(ctx, dt, NB, NB, am, an)
        B = dp.block_cyclic(ctx, dt, NB, NB, bm, bn)
        C = dp.block_cyclic(ctx, dt, NB, NB, M, N)
        dp.plrnt(ctx, A, 3872)
        dp.plrnt(ctx, B, 4674)
        dp.plrnt(ctx, C, 2873)
        dp.gemm(ctx, ta, tb, 0.51, A, B, -0.42, C)
        res.append(C.to_dense_local())
    assert rel_err(res[0], res[1]) < tol(dt)


def test_gemm_generic_path_matches_mfma(gctx):
    M = 384
    outs = []
    for gen in (False, True):
        ops.FORCE_GENERIC_GEMM = gen
        A = dp.block_cyclic(gctx, torch.float64, 128, 128, M, M)
        B = dp.block_cyclic(gctx, torch.float64, 128, 128, M, M)
        C = dp.block_cyclic(gctx, torch.float64, 128, 128, M, M)
        dp.plrnt(gctx, A, 1)
        dp.plrnt(gctx, B, 2)
        dp.gemm(gctx, 111, 112, 1.0, A, B, 0.0, C)
        outs.append(C.to_dense_local())
    ops.FORCE_GENERIC_GEMM = False
    assert rel_err(outs[0], outs[1]) < 1e-13


def test_mfma_layout_identity(gctx):
    """A = I with an asymmetric B catches transposed accumulator layouts."""
    n = 256
    A = dp.block_cyclic(gctx, torch.float64, n, n, n, n)
    B = dp.block_cyclic(gctx, torch.float64, n, n, n, n)
    C = dp.block_cyclic(gctx, torch.float64, n, n, n, n)
    A.from_dense(torch.eye(n, dtype=torch.float64))
    b = torch.arange(n * n, dtype=torch.float64).view(n, n) * 0.001 + torch.arange(n).view(n, 1) * 7.0
    B.from_dense(b)
    dp.gemm(gctx, 111, 111, 1.0, A, B, 0.0, C)
    assert torch.equal(C.to_dense_local(), b)


@pytest.mark.parametrize("prec", list("sdcz"))
@pytest.mark.parametrize("side", [dp.dplasmaLeft, dp.dplasmaRight])
@pytest.mark.parametrize("uplo", [dp.dplasmaLower, dp.dplasmaUpper])
@pytest.mark.parametrize("trans", [dp.dplasmaNoTrans, dp.dplasmaTrans, dp.dplasmaConjTrans])
@pytest.mark.parametrize("diag", [dp.dplasmaNonUnit, dp.dplasmaUnit])
def test_trsm_tile(gctx, cctx, prec, side, uplo, trans, diag):
    dt = DTYPES[prec]
    m, n = 150, 93
    k = m if side == dp.dplasmaLeft else n
    outs = []
    for ctx in (gctx, cctx):
        T = dp.block_cyclic(ctx, dt, k, k, k, k)
        dp.plghe(ctx, float(k), dp.dplasmaUpperLower, T, 11)  # well conditioned
        B = dp.block_cyclic(ctx, dt, m, n, m, n)
        dp.plrnt(ctx, B, 12)
        tb = TileBatch().add(0, m, n, b_off=0)
        ops.trsm(side, uplo, trans, diag, 0.7, T.data, T.ld, B.data, B.ld, tb)
        outs.append(B.to_dense_local())
    assert rel_err(outs[0], outs[1]) < tol(dt) * 10


@pytest.mark.parametrize("prec", list("sdcz"))
@pytest.mark.parametrize("uplo", [dp.dplasmaLower, dp.dplasmaUpper])
@pytest.mark.parametrize("dims", [(378, 93), (1024, 256), (600, 512)])
def test_potrf(gctx, prec, uplo, dims):
    dt = DTYPES[prec]
    N, NB = dims
    A = dp.block_cyclic(gctx, dt, NB, NB, N, N)
    dp.plghe(gctx, float(N), uplo, A, 3872)
    A0 = A.like()
    dp.lacpy(gctx, dp.dplasmaUpperLower, A, A0)
    info = dp.potrf(gctx, uplo, A)
    assert info == 0
    ok, res = dp.check_potrf(gctx, uplo, A, A0)
    assert ok, res


@pytest.mark.parametrize("uplo", [dp.dplasmaLower, dp.dplasmaUpper])
@pytest.mark.parametrize("N,NB,defer", [(3072, 256, 4), (2900, 256, 3), (6144, 512, 4)])
def test_potrf_deferred_blocks(gctx, uplo, N, NB, defer, monkeypatch):
    """Deferred trailing updates (blocks of D panels, k = D*NB) incl. a ragged last tile."""
    monkeypatch.setenv("DPLASMA_POTRF_DEFER", str(defer))
    monkeypatch.setenv("DPLASMA_POTRF_DEFER_MIN_TILES", "3")
    A = dp.block_cyclic(gctx, torch.float64, NB, NB, N, N)
    dp.plghe(gctx, float(N), uplo, A, 3872)
    A0 = A.like()
    dp.lacpy(gctx, dp.dplasmaUpperLower, A, A0)
    tp = dp.potrf_New(gctx, uplo, A)
    assert any(t.name.startswith("REST(") for t in tp.tasks)
    assert tp.execute(gctx) == 0
    ok, res = dp.check_potrf(gctx, uplo, A, A0)
    assert ok, res


def test_potrf_matches_cpu(gctx, cctx):
    N, NB = 700, 128
    outs = []
    for ctx in (gctx, cctx):
        A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
        dp.plghe(ctx, float(N), dp.dplasmaLower, A, 3872)
        dp.potrf(ctx, dp.dplasmaLower, A)
        outs.append(A.to_dense_local().tril())
    assert rel_err(outs[0], outs[1]) < 1e-12


def test_potrf_info_gpu(gctx):
    N, NB = 256, 64
    A = dp.block_cyclic(gctx, torch.float64, NB, NB, N, N)
    dp.plghe(gctx, 0.0, dp.dplasmaLower, A, 1)
    assert dp.potrf(gctx, dp.dplasmaLower, A) > 0


@pytest.mark.parametrize("norm", [dp.dplasmaMaxNorm, dp.dplasmaOneNorm, dp.dplasmaInfNorm, dp.dplasmaFrobeniusNorm])
def test_norms(gctx, cctx, norm):
    vals = []
    for ctx in (gctx, cctx):
        A = dp.block_cyclic(ctx, torch.complex128, 40, 40, 130, 130)
        dp.plghe(ctx, 2.0, dp.dplasmaUpperLower, A, 9)
        vals.append((dp.lange(ctx, norm, A), dp.lanhe(ctx, norm, dp.dplasmaLower, A)))
    assert abs(vals[0][0] - vals[1][0]) <= 1e-12 * vals[1][0]
    assert abs(vals[0][1] - vals[1][1]) <= 1e-12 * vals[1][1]


def test_lapack_storage_gemm(gctx, cctx):
    outs = []
    for ctx in (gctx, cctx):
        A = dp.block_cyclic(ctx, torch.float64, 64, 64, 200, 150, storage=dp.STORAGE_LAPACK, lld=203)
        B = dp.block_cyclic(ctx, torch.float64, 64, 64, 150, 170, storage=dp.STORAGE_LAPACK)
        C = dp.block_cyclic(ctx, torch.float64, 64, 64, 200, 170)
        dp.plrnt(ctx, A, 1)
        dp.plrnt(ctx, B, 2)
        dp.plrnt(ctx, C, 3)
        dp.gemm(ctx, 111, 111, 1.5, A, B, 0.5, C)
        outs.append(C.to_dense_local())
    assert rel_err(outs[0], outs[1]) < 1e-12


def test_blas3_gpu_matches_cpu(gctx, cctx):
    outs = []
    for ctx in (gctx, cctx):
        r = {}
        A = dp.block_cyclic(ctx, torch.float64, 64, 64, 300, 300)
        dp.plghe(ctx, 300.0, dp.dplasmaUpperLower, A, 3)
        for side in (141, 142):
            for uplo in (121, 122):
                for trans in (111, 113):
                    B = dp.block_cyclic(ctx, torch.float64, 64, 64, 300, 200) if side == 141 else \
                        dp.block_cyclic(ctx, torch.float64, 64, 64, 200, 300)
                    dp.plrnt(ctx, B, 4)
                    dp.trsm(ctx, side, uplo, trans, 131, 0.5, A, B)
                    r[("trsm", side, uplo, trans)] = B.to_dense_local()
                    dp.plrnt(ctx, B, 4)
                    dp.trmm(ctx, side, uplo, trans, 132, 0.5, A, B)
                    r[("trmm", side, uplo, trans)] = B.to_dense_local()
        A2 = dp.block_cyclic(ctx, torch.complex128, 64, 64, 256, 256)
        dp.plghe(ctx, 256.0, dp.dplasmaUpperLower, A2, 5)
        assert dp.poinv(ctx, dp.dplasmaLower, A2) == 0
        r["poinv"] = A2.to_dense_local().tril()
        C = dp.block_cyclic(ctx, torch.complex128, 64, 64, 256, 100)
        dp.plrnt(ctx, C, 6)
        D = dp.block_cyclic(ctx, torch.complex128, 64, 64, 256, 256)
        dp.herk(ctx, dp.dplasmaLower, dp.dplasmaNoTrans, 1.0, C, 0.0, D)
        r["herk"] = D.to_dense_local().tril()
        outs.append(r)
    for k in outs[1]:
        assert rel_err(outs[0][k], outs[1][k]) < 1e-10, k


@pytest.mark.parametrize("prec", list("sdz"))
def test_lu_gpu(gctx, cctx, prec):
    dt = DTYPES[prec]
    N, NB = 300, 64
    outs = []
    for ctx in (gctx, cctx):
        A = dp.block_cyclic(ctx, dt, NB, NB, N, N)
        dp.plrnt(ctx, A, 3872)
        IPIV = dp.ipiv_descriptor(ctx, A)
        assert dp.getrf_1d(ctx, A, IPIV) == 0
        B = dp.block_cyclic(ctx, dt, NB, NB, N, N)
        dp.plghe(ctx, float(N), dp.dplasmaUpperLower, B, 5)
        assert dp.getrf_nopiv(ctx, B) == 0
        outs.append((A.to_dense_local(), B.to_dense_local()))
    assert rel_err(outs[0][0], outs[1][0]) < tol(dt) * 100
    assert rel_err(outs[0][1], outs[1][1]) < tol(dt) * 100


@pytest.mark.parametrize("side,inplace", [("0", "1"), ("0", "0"), ("1", "1")])
def test_getrf_side_swaps(gctx, cctx, side, inplace, monkeypatch):
    """Partial-pivoting LU with the left-column interchanges on the side stream (opt-in) or not,
    row moves in place (k_rows_permute, default on one process) or staged (k_rows_move): same
    factors and pivots as the CPU path."""
    monkeypatch.setenv("DPLASMA_LU_SIDE_SWAPS", side)
    monkeypatch.setenv("DPLASMA_LU_INPLACE_MOVES", inplace)
    N, NB = 1100, 128
    outs = []
    for ctx in (gctx, cctx):
        A = dp.block_cyclic(ctx, torch.float64, NB, NB, N, N)
        dp.plrnt(ctx, A, 3872)
        IPIV = dp.ipiv_descriptor(ctx, A)
        assert dp.getrf_1d(ctx, A, IPIV) == 0
        outs.append((A.to_dense_local(), IPIV.to_dense_local()))
    assert torch.equal(outs[0][1].cpu(), outs[1][1].cpu())
    assert rel_err(outs[0][0], outs[1][0]) < 1e-11


@pytest.mark.parametrize("prec", list("sd"))
@pytest.mark.parametrize("ta,tb", [(111, 111), (111, 112), (112, 111), (112, 112)])
@pytest.mark.parametrize("mask,alpha,beta", [(0, -1.0, 1.0), (1, -1.0, 1.0), (2, 0.5, -0.3), (0, 2.0, 0.0)])
def test_gemm_full_tile_path(gctx, prec, ta, tb, mask, alpha, beta):
    """Whole-128-sub-tile batches take the branch-free buffer-load kernel (k_gemm_full): check it
    against torch for every transpose pair, triangular write masks and alpha/beta folding."""
    from dplasma_amd.ops.batch import GemmBatch
    dt = DTYPES[prec]
    nb, kt = 256, 3
    torch.manual_seed(7)
    A = torch.randn(nb * kt * nb, dtype=dt, device="cuda")       # kt tiles nb x nb, ld = nb
    B = torch.randn(nb * kt * nb, dtype=dt, device="cuda")
    C = torch.randn(2 * nb * nb, dtype=dt, device="cuda")        # 2 tiles
    C0 = C.clone()
    gb = GemmBatch()
    for t in range(2):
        gb.add(t * nb * nb, nb, nb, [(q * nb * nb, ((q + t) % kt) * nb * nb, nb) for q in range(kt)], mask)
    assert gb.full
    ops.gemm(ta, tb, alpha, A, nb, B, nb, beta, C, nb, gb)
    torch.cuda.synchronize()

    def tile(X, i):
        return X[i * nb * nb:(i + 1) * nb * nb].view(nb, nb).t().double()   # column-major view
    for t in range(2):
        acc = torch.zeros(nb, nb, dtype=torch.float64, device="cuda")
        for q in range(kt):
            a = tile(A, q) if ta == 111 else tile(A, q).t()
            b = tile(B, (q + t) % kt) if tb == 111 else tile(B, (q + t) % kt).t()
            acc += a @ b
        ref = beta * tile(C0, t) + alpha * acc
        keep = tile(C0, t)
        if mask == 1:
            ref = torch.where(torch.ones(nb, nb, dtype=torch.bool, device="cuda").tril(), ref, keep)
        elif mask == 2:
            ref = torch.where(torch.ones(nb, nb, dtype=torch.bool, device="cuda").triu(), ref, keep)
        got = tile(C, t)
        assert (got - ref).abs().max().item() / ref.abs().max().item() < (1e-12 if prec == "d" else 1e-4)


@pytest.mark.parametrize("m,n", [(2000, 128), (4096, 512), (1500, 200), (512, 512), (300, 512), (70000, 128),
                                 (40000, 64)])
def test_panel_lu_device(gctx, m, n):
    """Recursive device-resident panel LU (<=64-column blocks with the multi-workgroup on-device
    pivot search) against LAPACK partial pivoting (torch.linalg.lu_factor on the CPU)."""
    torch.manual_seed(3)
    ld = m
    a = torch.randn(m, n, dtype=torch.float64)
    P = a.t().contiguous().view(-1).cuda()          # column-major
    ipiv = torch.zeros(n, dtype=torch.int32, device="cuda")
    ws = ops.lu_workspace(m, "cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    info = torch.zeros(1, dtype=torch.int32, device="cuda")
    plu = ops.PanelLU(P, ld, m, n)
    plu.run(ipiv, ws, cnt, info, 0)
    torch.cuda.synchronize()
    k = min(m, n)
    LU_ref, piv_ref = torch.linalg.lu_factor(a)
    got = P.view(n, m).t().cpu()
    assert torch.equal(ipiv[:k].cpu().long(), piv_ref[:k].long() - 1)
    assert (got - LU_ref).abs().max().item() < 1e-10 * max(1.0, LU_ref.abs().max().item())
    assert int(info.item()) == 0


def test_piv_moves_device(gctx):
    """Sequential interchanges -> net row moves, on the device vs the host fallback."""
    torch.manual_seed(5)
    kb, mp = 512, 5000
    piv = torch.tensor([int(torch.randint(i, mp, (1,))) for i in range(kb)], dtype=torch.int32)
    outs = []
    for dev in ("cuda", "cpu"):
        d = torch.zeros(2 * kb, dtype=torch.int32, device=dev)
        s = torch.zeros(2 * kb, dtype=torch.int32, device=dev)
        c = torch.zeros(1, dtype=torch.int32, device=dev)
        ops.piv_moves(piv.to(dev), kb, d, s, c)
        n = int(c[0])
        outs.append(sorted(zip(d[:n].cpu().tolist(), s[:n].cpu().tolist())))
    assert outs[0] == outs[1]


@pytest.mark.parametrize("prec", list("dz"))
@pytest.mark.parametrize("seg", [(0, 64), (64, 320), (100, 356), (0, 600)])
def test_laswp_panel_device(gctx, prec, seg):
    """Panel interchanges on the device (content-parallel net moves; > 512 swaps: sequential
    fallback) vs the host replay of the same LAPACK ipiv segment."""
    torch.manual_seed(7)
    i0, i1 = seg
    m, ld, ncols = 3000, 3008, 77
    ipiv = torch.tensor([int(torch.randint(i, min(m, i + (4 if i % 3 else m)), (1,))) for i in range(i1)],
                        dtype=torch.int32)
    P = torch.randn(ld * (ncols + 3), dtype=DTYPES[prec])
    outs = []
    for dev in ("cuda", "cpu"):
        X = P.clone().to(dev)
        ops.laswp_panel(X, ld, 2, 2 + ncols, ipiv.to(dev), i0, i1)
        outs.append(X.cpu())
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("prec", list("dz"))
@pytest.mark.parametrize("uplo", [dp.dplasmaLower, dp.dplasmaUpper])
@pytest.mark.parametrize("dims", [(1024, 512), (1100, 300)])
def test_potrf_blocked_tile_kernel(gctx, prec, uplo, dims, monkeypatch):
    """Diagonal tiles as 128-wide POTRF + TRSM + masked MFMA GEMM steps (distributed default)."""
    monkeypatch.setenv("DPLASMA_POTRF_TILE", "blocked")
    dt = DTYPES[prec]
    N, NB = dims
    A = dp.block_cyclic(gctx, dt, NB, NB, N, N)
    dp.plghe(gctx, float(N), uplo, A, 3872)
    A0 = A.like()
    dp.lacpy(gctx, dp.dplasmaUpperLower, A, A0)
    assert dp.potrf(gctx, uplo, A) == 0
    ok, res = dp.check_potrf(gctx, uplo, A, A0)
    assert ok, res


@pytest.mark.parametrize("prec", list("sd"))
@pytest.mark.parametrize("ta,tb", [(111, 111), (111, 112), (112, 111), (112, 112)])
@pytest.mark.parametrize("cap", [8, 24])
def test_gemm_full_capped_grid(gctx, prec, ta, tb, cap):
    """Capped grid-stride k_gemm_full (ops.gemm_wg_cap, the bulk-update mode that keeps CUs free for
    the critical path): each workgroup walks several sub-tiles; the result is bit-identical to the
    one-sub-tile-per-workgroup launch (same per-tile arithmetic), triangle masks included."""
    from dplasma_amd.ops.batch import GemmBatch
    dt = DTYPES[prec]
    nb, kt = 512, 2
    torch.manual_seed(11)
    A = torch.randn(nb * kt * nb, dtype=dt, device="cuda")
    B = torch.randn(nb * kt * nb, dtype=dt, device="cuda")
    C = torch.randn(3 * nb * nb, dtype=dt, device="cuda")
    gb = GemmBatch()
    for t in range(3):
        gb.add(t * nb * nb, nb, nb, [(q * nb * nb, ((q + t) % kt) * nb * nb, nb) for q in range(kt)], t % 2)
    assert gb.full
    ref = C.clone()
    ops.gemm(ta, tb, -1.0, A, nb, B, nb, 1.0, ref, nb, gb)
    with ops.gemm_wg_cap(cap):
        ops.gemm(ta, tb, -1.0, A, nb, B, nb, 1.0, C, nb, gb)
    assert _lib.load().dpl_gemm_set_wg_cap(0) == 0      # the context manager restored "uncapped"
    torch.cuda.synchronize()
    assert torch.equal(C, ref)


@pytest.mark.parametrize("prec", list("sdcz"))
@pytest.mark.parametrize("storage", [dp.STORAGE_TILE, dp.STORAGE_LAPACK])
def test_swap_transpose(gctx, cctx, prec, storage):
    """ops.swap_transpose (HIP) vs the CPU reference: ragged tiles, in-place diagonal tiles, conj."""
    from dplasma_amd.ops import tile_ops
    from dplasma_amd.ops.batch import TileBatch
    dt = DTYPES[prec]
    G, C = _pair(gctx, cctx, dt, 96, 96, 333, 333, storage=storage)
    dp.plrnt(gctx, G, 7)
    dp.plrnt(cctx, C, 7)
    for M in (G, C):
        xb = TileBatch()
        for j in range(M.nt):
            for i in range(j, M.mt):
                xb.add(M.offset(i, j), M.tile_rows(i), M.tile_cols(j), b_off=M.offset(j, i))
        tile_ops.swap_transpose(M.data, M.ld, xb, conj=dt.is_complex)
    g, c = G.to_dense_local().cpu(), C.to_dense_local()
    assert torch.equal(g, c)
    d0 = dp.block_cyclic(cctx, dt, 96, 96, 333, 333, storage=storage)
    dp.plrnt(cctx, d0, 7)
    ref = d0.to_dense_local().t()
    assert torch.equal(c, ref.conj() if dt.is_complex else ref)
    # one-way copy: Y's upper tiles <- op(X's lower tiles)^T, diagonal tiles upper part only
    X, Y = _pair(gctx, cctx, dt, 96, 96, 333, 333, storage=storage)[0], G
    dp.plrnt(gctx, X, 9)
    y0 = Y.to_dense_local().clone()
    xb, db = TileBatch(), TileBatch()
    for j in range(X.nt):
        for i in range(j, X.mt):
            (db if i == j else xb).add(X.offset(i, j), X.tile_rows(i), X.tile_cols(j), b_off=Y.offset(j, i))
    tile_ops.copy_transpose(X.data, X.ld, Y.data, Y.ld, xb, conj=dt.is_complex)
    tile_ops.copy_transpose(X.data, X.ld, Y.data, Y.ld, db, conj=dt.is_complex, upper_only=True)
    xt = X.to_dense_local().t()
    xt = xt.conj() if dt.is_complex else xt
    y = Y.to_dense_local()
    assert torch.equal(torch.triu(y), torch.triu(xt)) and torch.equal(torch.tril(y, -1), torch.tril(y0, -1))


@pytest.mark.parametrize("dims", [(378, 93), (2048, 512)])
def test_potrf_upper_via_lower_gpu(gctx, dims, monkeypatch):
    """Upper DPOTRF on one GPU runs the transposed lower schedule: residual and untouched lower part."""
    N, NB = dims
    monkeypatch.setenv("DPLASMA_POTRF_UPPER", "auto")
    A = dp.block_cyclic(gctx, torch.float64, NB, NB, N, N)
    dp.plghe(gctx, float(N), dp.dplasmaUpperLower, A, 3872)
    A0 = A.like()
    dp.lacpy(gctx, dp.dplasmaUpperLower, A, A0)
    low0 = torch.tril(A0.to_dense_local(), -1).cpu()
    assert dp.dpotrf(gctx, dp.dplasmaUpper, A) == 0
    ok, res = dp.check_potrf(gctx, dp.dplasmaUpper, A, A0)
    assert ok, res
    assert torch.equal(torch.tril(A.to_dense_local(), -1).cpu(), low0)
