"""Matrix generators: LCG skip-ahead semantics and distribution independence."""
import numpy as np
import pytest
import torch

import dplasma_amd as dp
from dplasma_amd.utils import lcg

MASK = (1 << 64) - 1


def ref_jump(n, seed):
    a, c, ran = 6364136223846793005, 1, seed
    while n:
        if n & 1:
            ran = (a * ran + c) & MASK
        c = (c * (a + 1)) & MASK
        a = (a * a) & MASK
        n >>= 1
    return ran


def ref_val(ran):
    return float(np.float32(0.5) - np.float32(ran) * np.float32(5.4210108624275222e-20))


def test_jump_matches_scalar_reference():
    idx = np.array([0, 1, 2, 17, 1000, 123456789, 2**40 + 3], dtype=np.uint64)
    got = lcg.jump(idx, 3872)
    for i, n in enumerate(idx):
        assert int(got[i]) == ref_jump(int(n), 3872)


def test_sequential_equals_jump():
    # the value at i+1 is one LCG step after the value at i
    r0 = ref_jump(5, 42)
    r1 = (6364136223846793005 * r0 + 1) & MASK
    assert r1 == ref_jump(6, 42)


def test_plrnt_values():
    blk = lcg.rnd_block(3, 2, 4, 5, 50, 3872, False)
    for i in range(4):
        for j in range(5):
            assert blk[i, j] == ref_val(ref_jump((3 + i) + (2 + j) * 50, 3872))


def test_plrnt_complex_values():
    blk = lcg.rnd_block(0, 1, 3, 2, 10, 7, True)
    for i in range(3):
        for j in range(2):
            r = ref_jump(2 * (i + (1 + j) * 10), 7)
            r2 = (6364136223846793005 * r + 1) & MASK
            assert blk[i, j] == complex(ref_val(r), ref_val(r2))


@pytest.mark.parametrize("prec", ["d", "z"])
def test_plghe_hermitian_and_tiling_independent(prec):
    ctx = dp.init(device="cpu")
    dt = dp.PREC_DTYPE[prec]
    N = 57
    mats = []
    for nb in (7, 13, 57):
        A = dp.block_cyclic(ctx, dt, nb, nb, N, N)
        dp.plghe(ctx, float(N), dp.dplasmaUpperLower, A, 3872)
        mats.append(A.to_dense_local())
    assert torch.equal(mats[0], mats[1]) and torch.equal(mats[0], mats[2])
    M = mats[0]
    assert torch.allclose(M, M.conj().T)
    assert (torch.diagonal(M).real > N - 1).all()


def test_plrnt_storage_independent():
    ctx = dp.init(device="cpu")
    A = dp.block_cyclic(ctx, torch.float64, 10, 10, 33, 21)
    B = dp.block_cyclic(ctx, torch.float64, 10, 10, 33, 21, storage=dp.STORAGE_LAPACK)
    dp.plrnt(ctx, A, 99)
    dp.plrnt(ctx, B, 99)
    assert torch.equal(A.to_dense_local(), B.to_dense_local())
