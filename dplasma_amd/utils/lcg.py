"""Host (CPU) reference of the matrix generators, bit-identical to the GPU ones.

Implements the PLASMA 64-bit LCG with O(log n) skip-ahead used by the
reference (``src/cores/random.h:20-41``; element value ``0.5f - ran*RndF_Mul``
in float arithmetic, ``src/cores/core_zplrnt.c:68-91``).  The value of element
(I, J) depends only on its global position, so any distribution/tiling gives
the same matrix.  Vectorised with numpy uint64 (wrap-around arithmetic).
"""
from __future__ import annotations

import numpy as np

A = np.uint64(6364136223846793005)
C = np.uint64(1)
RNDF_MUL = np.float32(5.4210108624275222e-20)

# precomputed (a_k, c_k) for each bit: applying bit i = x -> a_k*x + c_k
_AK = []
_CK = []
_a, _c = A, C
with np.errstate(over="ignore"):
    for _ in range(64):
        _AK.append(_a)
        _CK.append(_c)
        _c = np.uint64(_c * (_a + np.uint64(1)))
        _a = np.uint64(_a * _a)


def jump(n: np.ndarray, seed: int) -> np.ndarray:
    """Vectorised Rnd64_jump(n, seed)."""
    n = np.asarray(n, dtype=np.uint64).copy()
    ran = np.full(n.shape, np.uint64(seed), dtype=np.uint64)
    with np.errstate(over="ignore"):
        for i in range(64):
            if not n.any():
                break
            bit = (n & np.uint64(1)).astype(bool)
            ran = np.where(bit, ran * _AK[i] + _CK[i], ran)
            n >>= np.uint64(1)
    return ran


def _val(ran: np.ndarray) -> np.ndarray:
    return (np.float32(0.5) - ran.astype(np.float32) * RNDF_MUL).astype(np.float32)


def rnd_block(I0: int, J0: int, m: int, n: int, gM: int, seed: int, complex_: bool) -> np.ndarray:
    """Values of the plrnt stream on global rows I0..I0+m-1, cols J0..J0+n-1."""
    I = np.arange(I0, I0 + m, dtype=np.uint64)[:, None]
    J = np.arange(J0, J0 + n, dtype=np.uint64)[None, :]
    idx = I + J * np.uint64(gM)
    if not complex_:
        return _val(jump(idx, seed)).astype(np.float64)
    r = jump(np.uint64(2) * idx, seed)
    with np.errstate(over="ignore"):
        r2 = r * A + C
    return _val(r).astype(np.float64) + 1j * _val(r2).astype(np.float64)


def generate_block(kind: str, I0: int, J0: int, m: int, n: int, gM: int, seed: int, complex_: bool,
                   bump=0.0) -> np.ndarray:
    """Block (I0:I0+m, J0:J0+n) of plrnt ('rnt'), plghe ('ghe') or plgsy ('gsy')."""
    if kind == "rnt":
        return rnd_block(I0, J0, m, n, gM, seed, complex_)
    I = np.arange(I0, I0 + m)[:, None]
    J = np.arange(J0, J0 + n)[None, :]
    low = rnd_block(I0, J0, m, n, gM, seed, complex_)
    # transposed stream: value at (J, I)
    up = rnd_block(J0, I0, n, m, gM, seed, complex_).T
    if kind == "ghe":
        up = np.conj(up)
    out = np.where(I > J, low, up)
    d = (I == J)
    if d.any():
        if kind == "ghe":
            diag = np.real(low) + np.real(bump)
        else:
            diag = low + bump
        out = np.where(d, diag, out)
    return out
