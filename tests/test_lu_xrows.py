"""Point-to-point row interchanges between process rows (models/lu.py _xswap; the reference's SWAP_COLLECT /
SWAP_SND, src/zgetrf_ptgpanel.jdf:825-984): the move classifier and the pack / unpack copies.

CPU: the classes and ordinals agree between sender and receiver for every pair of process rows, and a full
exchange simulated between P "ranks" reproduces the one-process permutation.  GPU: the HIP kernels
(k_rows_xord, k_rows_xcopy in csrc/kernels/lu_piv.hip) equal the CPU path of the same op."""
import numpy as np
import pytest
import torch

from dplasma_amd.ops import tile_ops as ops


def _moves(kb, mrel, seed):
    g = np.random.default_rng(seed)
    piv = np.array([g.integers(i, mrel) for i in range(kb)], dtype=np.int32)
    dst = torch.zeros(2 * kb, dtype=torch.int32)
    src = torch.zeros(2 * kb, dtype=torch.int32)
    cnt = torch.zeros(1, dtype=torch.int32)
    ops.piv_moves(torch.from_numpy(piv), kb, dst, src, cnt, mrel=mrel)
    return piv, dst, src, cnt


@pytest.mark.parametrize("P,seed", [(2, 0), (2, 1), (3, 2), (4, 3)])
def test_xrows_exchange_equals_permutation(P, seed):
    mb, kb, mt, k = 8, 8, 12, 2
    r0 = k * mb
    mrel = mt * mb - r0
    piv, dst, src, cnt = _moves(kb, mrel, seed)
    prow = torch.tensor([m % P for m in range(mt)], dtype=torch.int32)
    W = 5
    full = torch.randn(mt * mb, W, dtype=torch.float64)
    ref = full.clone()
    for i, p in enumerate(piv):          # sequential interchanges (LAPACK laswp)
        a, b = r0 + i, r0 + int(p)
        ref[[a, b]] = ref[[b, a]]
    n = int(cnt[0])
    xo = {q: torch.full((2 * kb,), -1, dtype=torch.int32) for q in range(P)}
    for q in range(P):
        ops.rows_xord(dst, src, cnt, r0, mb, prow, q, P, kb, xo[q])
    # every rank stages its own source rows (slot-major, ldb = 2 kb), packs, "sends", unpacks, scatters
    ldb = 2 * kb
    own = lambda R, q: int(prow[R // mb]) == q  # noqa: E731
    tmp = {}
    sendb = {q: [torch.zeros(kb * W, dtype=torch.float64) for _ in range(P)] for q in range(P)}
    for q in range(P):
        t = torch.zeros(ldb * W, dtype=torch.float64)
        for s in range(n):
            R = r0 + int(src[s])
            if own(R, q):
                t[s::ldb][:W] = full[R]
        tmp[q] = t
        ops.rows_xcopy(True, t, ldb, W, xo[q], cnt, ldb, sendb[q], kb)
    out = full.clone()
    for q in range(P):
        recvb = [sendb[p][q] if p != q else None for p in range(P)]   # what p packed for q
        ops.rows_xcopy(False, tmp[q], ldb, W, xo[q], cnt, ldb, recvb, kb)
        for s in range(n):
            R = r0 + int(dst[s])
            if own(R, q):
                out[R] = tmp[q][s::ldb][:W]
    assert torch.equal(out, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("P,me", [(2, 0), (2, 1), (4, 2)])
def test_gpu_xrows_kernels_match_cpu(P, me):
    from dplasma_amd.ops import _lib
    _lib.load(build_if_missing=False)
    mb, kb, mt, k = 512, 512, 40, 3
    r0 = k * mb
    mrel = mt * mb - r0
    piv, dst, src, cnt = _moves(kb, mrel, 11 + me)
    prow = torch.tensor([m % P for m in range(mt)], dtype=torch.int32)
    xo_c = torch.full((2 * kb,), -1, dtype=torch.int32)
    ops.rows_xord(dst, src, cnt, r0, mb, prow, me, P, kb, xo_c)
    dev = torch.device("cuda", 0)
    xo_g = torch.full((2 * kb,), -1, dtype=torch.int32, device=dev)
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    ops.rows_xord(dst.to(dev), src.to(dev), cnt.to(dev), r0, mb, prow.to(dev), me, P, kb, xo_g, info)
    n = int(cnt[0])
    assert torch.equal(xo_g.cpu()[:n], xo_c[:n]) and int(info) == 0
    ldb, W = 2 * kb, 700
    tmp = torch.randn(ldb * W, dtype=torch.float64)
    bufs_c = [torch.zeros(kb * W, dtype=torch.float64) if q != me else None for q in range(P)]
    ops.rows_xcopy(True, tmp, ldb, W, xo_c, cnt, ldb, bufs_c, kb)
    tmp_g = tmp.to(dev)
    bufs_g = [torch.zeros(kb * W, dtype=torch.float64, device=dev) for _ in range(P)]
    ptrs = torch.tensor([b.data_ptr() for b in bufs_g], dtype=torch.int64, device=dev)
    ops.rows_xcopy(True, tmp_g, ldb, W, xo_g, cnt.to(dev), ldb, ptrs, kb)
    for q in range(P):
        if q != me:
            assert torch.equal(bufs_g[q].cpu(), bufs_c[q])
    # unpack: arriving rows land in their staging slots
    src_b = [torch.randn(kb * W, dtype=torch.float64) if q != me else None for q in range(P)]
    t_c = tmp.clone()
    ops.rows_xcopy(False, t_c, ldb, W, xo_c, cnt, ldb, src_b, kb)
    t_g = tmp.to(dev)
    sb_g = [b.to(dev) if b is not None else torch.zeros(1, dtype=torch.float64, device=dev) for b in src_b]
    ptrs = torch.tensor([b.data_ptr() for b in sb_g], dtype=torch.int64, device=dev)
    ops.rows_xcopy(False, t_g, ldb, W, xo_g, cnt.to(dev), ldb, ptrs, kb)
    torch.cuda.synchronize()
    assert torch.equal(t_g.cpu(), t_c)
