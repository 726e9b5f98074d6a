"""Batched tile operations: one entry point per CORE kernel family.

Each function takes base tensors (a descriptor's local storage or a panel
buffer), leading dimensions and an item batch, and runs either

* the native HIP/CDNA4 kernel (``lib/libdplasma_kernels.so``) on the current
  torch stream when the data lives on a GPU -- a single launch per batch; or
* the CPU reference path (PyTorch CPU ops on tile views -- the analogue of the
  reference's ``CORE_z*`` CBLAS/LAPACKE wrappers, ``src/cores/core_zgemm.c:90``,
  ``core_zpotrf.c:68`` ...) when the data lives in host memory.

GPU tensors never fall back to PyTorch/rocBLAS: a missing or failing kernel
raises.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch

from ..constants import (dplasmaConjTrans, dplasmaLeft, dplasmaLower, dplasmaNonUnit, dplasmaNoTrans, dplasmaRight,
                         dplasmaTrans, dplasmaUnit, dplasmaUpper)
from ..utils import lcg
from . import _lib
from .batch import _pred as _pred_items
from .batch import MASK_LOWER, MASK_UPPER, GemmBatch, TileBatch

FORCE_GENERIC_GEMM = False  # testing knob: route real GEMMs through the FMA kernel


def _view(base: torch.Tensor, off: int, rows: int, cols: int, ld: int) -> torch.Tensor:
    # offsets are relative to base's first element (as data_ptr() is for the GPU kernels)
    return torch.as_strided(base, (rows, cols), (1, ld), base.storage_offset() + int(off))


def _op(x: torch.Tensor, trans: int) -> torch.Tensor:
    if trans == dplasmaNoTrans:
        return x
    if trans == dplasmaTrans:
        return x.transpose(0, 1)
    return x.conj().transpose(0, 1)


def _is_gpu(t: torch.Tensor) -> bool:
    return t.device.type == "cuda"


# ----------------------------------------------------------------------------- GEMM
class gemm_wg_cap:
    """``with gemm_wg_cap(n):`` -- full-tile MFMA GEMM launches issued inside hold at most n workgroup
    slots (grid-stride over their sub-tiles; 0 = uncapped).  A bulk trailing update launched that way
    leaves CUs free for the latency-bound critical-path kernels of a high-priority stream
    (``dpl_gemm_set_wg_cap``, csrc/kernels/gemm.hip).  No effect on the CPU path."""

    def __init__(self, n: int):
        self.n = int(n)
        self.old = 0

    def __enter__(self):
        if self.n > 0 and torch.cuda.is_available():
            self.old = _lib.load().dpl_gemm_set_wg_cap(self.n)
        return self

    def __exit__(self, *exc):
        if self.n > 0 and torch.cuda.is_available():
            _lib.load().dpl_gemm_set_wg_cap(self.old)
        return False


def gemm(transA: int, transB: int, alpha, A: torch.Tensor, lda: int, B: torch.Tensor, ldb: int, beta,
         C: torch.Tensor, ldc: int, batch: GemmBatch):
    """For every item: C = beta*C + alpha * sum_k opA(A_k) opB(B_k) (masked to a triangle if asked)."""
    batch.finalize()
    if len(batch) == 0:
        return
    if _is_gpu(C):
        lib = _lib.load()
        items, kps = batch.device_arrays(C.device)
        ve = max(1, 16 // C.element_size())   # elements per 16-byte vector
        vec_ok = int(batch.aligned(ve) and lda % ve == 0 and ldb % ve == 0 and A.data_ptr() % 16 == 0
                     and B.data_ptr() % 16 == 0)
        if vec_ok and batch.full:
            vec_ok |= 2
        sa, sb = _lib.Scalar(alpha, C.dtype), _lib.Scalar(beta, C.dtype)
        rc = lib.dpl_gemm_batched(_lib.prec_code(C.dtype), transA, transB, len(batch.items), items.data_ptr(),
                                  kps.data_ptr(), batch.max_m, batch.max_n, sa.ptr, A.data_ptr(), lda, B.data_ptr(),
                                  ldb, sb.ptr, C.data_ptr(), ldc, vec_ok, int(FORCE_GENERIC_GEMM), _lib.stream_ptr())
        _lib.check(rc, "gemm_batched")
        return
    for it in batch.items:
        m, n = int(it["m"]), int(it["n"])
        c = _view(C, it["c_off"], m, n, ldc)
        acc = None
        for kp in batch.kpairs[it["kt_beg"]:it["kt_beg"] + it["kt_cnt"]]:
            k = int(kp["k"])
            a = _view(A, kp["a_off"], m, k, lda) if transA == dplasmaNoTrans else _op(_view(A, kp["a_off"], k, m, lda), transA)
            b = _view(B, kp["b_off"], k, n, ldb) if transB == dplasmaNoTrans else _op(_view(B, kp["b_off"], n, k, ldb), transB)
            p = a @ b
            acc = p if acc is None else acc + p
        new = c * beta if beta != 0 else torch.zeros_like(c)
        if acc is not None:
            new = new + alpha * acc
        mask = int(it["flags"]) & 3
        if mask == MASK_LOWER:
            new = torch.where(torch.ones(m, n, dtype=torch.bool).tril(), new, c)
        elif mask == MASK_UPPER:
            new = torch.where(torch.ones(m, n, dtype=torch.bool).triu(), new, c)
        c.copy_(new)


# ----------------------------------------------------------------------------- POTRF
def potrf_tile(uplo: int, A: torch.Tensor, off: int, n: int, lda: int, info: torch.Tensor, info_base: int,
               zbuf: torch.Tensor = None):
    """Cholesky of one diagonal tile in place; ``info`` (int32 tensor, 1 elem) gets base + first bad col.

    ``zbuf`` (fp64 GPU tiles with n <= 512, see :func:`rb_zbuf`): also receive the inverted
    diagonal 32-blocks for :func:`trsm_rb`."""
    if n <= 0:
        return
    if _is_gpu(A):
        lib = _lib.load()
        if zbuf is not None:
            assert rb_ok(A, n) and zbuf.dtype == torch.float64 and zbuf.numel() >= rb_zbuf_size()
            rc = lib.dpl_potrf_tile_rbz(uplo, n, A.data_ptr() + 8 * int(off), lda, info.data_ptr(), int(info_base),
                                        zbuf.data_ptr(), _lib.stream_ptr())
        else:
            rc = lib.dpl_potrf_tile(_lib.prec_code(A.dtype), uplo, n, A.data_ptr(), int(off), lda, info.data_ptr(),
                                    int(info_base), _lib.stream_ptr())
        _lib.check(rc, "potrf_tile")
        return
    t = _view(A, off, n, n, lda)
    upper = uplo == dplasmaUpper
    src = t.triu() if upper else t.tril()
    herm = src + _op(src, dplasmaConjTrans) - torch.diag_embed(torch.diagonal(src))
    if herm.is_complex():
        herm = herm - 1j * torch.diag_embed(torch.diagonal(herm).imag)
    L, inf = torch.linalg.cholesky_ex(herm, upper=upper)
    bad = int(inf)
    if bad > 0:
        if int(info[0]) == 0:
            info[0] = info_base + bad
        # mimic LAPACK: factor up to the failing column, keep what we have
    keep = torch.ones(n, n, dtype=torch.bool).triu() if upper else torch.ones(n, n, dtype=torch.bool).tril()
    t.copy_(torch.where(keep, L, t))


_POTRF_BLK_PLANS = {}


def _potrf_blocked_plan(uplo: int, n: int, lda: int, nb: int):
    """Sub-block batches of a right-looking tile Cholesky, offsets relative to the tile origin
    (so one plan serves every diagonal tile of the same size and leading dimension)."""
    key = (uplo, n, lda, nb)
    plan = _POTRF_BLK_PLANS.get(key)
    if plan is not None:
        return plan
    lower = uplo == dplasmaLower

    def at(i, j):  # sub-block (i, j) of the "lower" picture; upper stores its transpose
        return (i + j * lda) if lower else (j + i * lda)

    steps = []
    starts = list(range(0, n, nb))
    for jj, j0 in enumerate(starts):
        jb = min(nb, n - j0)
        below = starts[jj + 1:]
        tb = gb = None
        if below:
            tb = TileBatch()
            for i0 in below:
                ib = min(nb, n - i0)
                if lower:
                    tb.add(at(j0, j0), ib, jb, b_off=at(i0, j0))
                else:
                    tb.add(at(j0, j0), jb, ib, b_off=at(i0, j0))
            tb.finalize()
            gb = GemmBatch()
            for c0 in below:
                cb = min(nb, n - c0)
                for r0 in range(c0, n, nb):
                    rb = min(nb, n - r0)
                    mask = (MASK_LOWER if lower else MASK_UPPER) if r0 == c0 else 0
                    if lower:  # C(r, c) -= L(r, j) L(c, j)^H
                        gb.add(at(r0, c0), rb, cb, [(at(r0, j0), at(c0, j0), jb)], mask)
                    else:      # C(c, r) -= U(j, c)^H U(j, r)
                        gb.add(at(r0, c0), cb, rb, [(at(c0, j0), at(r0, j0), jb)], mask)
            gb.finalize()
        steps.append((j0, jb, tb, gb))
    plan = _POTRF_BLK_PLANS[key] = steps
    return plan


def potrf_tile_blocked(uplo: int, A: torch.Tensor, off: int, n: int, lda: int, info: torch.Tensor, info_base: int,
                       nb: int = 128):
    """Cholesky of one diagonal tile as nb-wide right-looking steps: single-workgroup POTRF of the
    nb x nb diagonal block, batched TRSM of the blocks below it, masked MFMA GEMM update of the
    rest.  Several workgroups per step instead of one: the critical-path tile factorisation of the
    distributed POTRF (where per-rank trailing updates are too small to hide a ~0.6 ms
    single-workgroup 512 x 512 factorisation) -- reference: the GPU potrf incarnation,
    ``src/zpotrf_L.jdf`` (cusolverDnXpotrf body)."""
    if n <= nb:
        return potrf_tile(uplo, A, off, n, lda, info, info_base)
    lower = uplo == dplasmaLower
    V = A.view(-1)[int(off):]
    tA, tB = (dplasmaNoTrans, dplasmaConjTrans) if lower else (dplasmaConjTrans, dplasmaNoTrans)
    side = dplasmaRight if lower else dplasmaLeft
    for j0, jb, tb, gb in _potrf_blocked_plan(uplo, n, lda, nb):
        potrf_tile(uplo, V, j0 + j0 * lda, jb, lda, info, info_base + j0)
        if tb is None:
            continue
        trsm(side, uplo, dplasmaConjTrans, dplasmaNonUnit, 1.0, V, lda, V, lda, tb)
        gemm(tA, tB, -1.0, V, lda, V, lda, 1.0, V, lda, gb)


# ----------------------------------------------------------------------------- POTRF panel TRSM (rb)
RB_ROWS = 16  # strip height of the panel TRSM kernel (csrc/kernels/potrf_rb.hip k_trsm_rb)
_RB_ITEM = np.dtype([("b_off", np.int64), ("rows", np.int32), ("pad", np.int32)])


def rb_ok(A: torch.Tensor, n: int) -> bool:
    """fp64 GPU tiles of order <= 512 use the dataflow POTRF / panel-TRSM kernels."""
    return _is_gpu(A) and A.dtype == torch.float64 and 0 < n <= 512


def rb_zbuf_size() -> int:
    return int(_lib.load().dpl_potrf_zbuf_size())


class RbPanel:
    """16-row strips of the panel tiles B_i (m_i x n) solved by :func:`trsm_rb`: for lower storage a
    strip is 16 consecutive rows of a tile (offset b_off + r); for upper storage (B_i = A(k, i),
    solved from the left) the same thing on the transposed view (16 consecutive columns)."""

    def __init__(self, uplo: int, tiles, ldb: int):
        rows = []
        for b_off, m in tiles:
            for r0 in range(0, m, RB_ROWS):
                off = b_off + (r0 if uplo == dplasmaLower else r0 * ldb)
                rows.append((off, min(RB_ROWS, m - r0), 0))
        self.items = np.array(rows, dtype=_RB_ITEM)
        self._dev = {}

    def __len__(self):
        return len(self.items)

    def device(self, dev):
        key = str(dev)
        t = self._dev.get(key)
        if t is None:
            t = self._dev[key] = torch.from_numpy(self.items.view(np.uint8).copy()).to(dev)
        return t


def potrf_trsm_rb(uplo: int, n: int, A: torch.Tensor, off: int, lda: int, info: torch.Tensor, info_base: int,
                  zbuf: torch.Tensor, panel: "RbPanel", B: torch.Tensor, ldb: int):
    """Fused diagonal-tile Cholesky + panel solve (k_potrf_trsm_rb): the tile at A[off] is factored
    and the strips of ``panel`` (in B) are solved along the factorisation wavefront in ONE launch."""
    assert rb_ok(A, n) and zbuf.dtype == torch.float64 and zbuf.numel() >= rb_zbuf_size()
    rc = _lib.load().dpl_potrf_trsm_rb(uplo, n, A.data_ptr() + 8 * int(off), lda, info.data_ptr(), int(info_base),
                                       zbuf.data_ptr(), len(panel), panel.device(B.device).data_ptr() if len(panel)
                                       else None, B.data_ptr(), ldb, _lib.stream_ptr())
    _lib.check(rc, "potrf_trsm_rb")


def trsm_rb_prep(uplo: int, n: int, L: torch.Tensor, l_off: int, ldl: int, zbuf: torch.Tensor):
    """Inverted diagonal 32-blocks of an already factored tile (ranks that received it)."""
    rc = _lib.load().dpl_trsm_rb_prep(uplo, n, L.data_ptr() + 8 * int(l_off), ldl, zbuf.data_ptr(),
                                      _lib.stream_ptr())
    _lib.check(rc, "trsm_rb_prep")


def trsm_rb(uplo: int, n: int, L: torch.Tensor, l_off: int, ldl: int, zbuf: torch.Tensor, panel: RbPanel,
            B: torch.Tensor, ldb: int):
    """Panel solve of the Cholesky step: B_i := B_i L^{-H} (lower) / U^{-H} B_i (upper) for every panel
    tile of ``panel``, L the factored n x n tile at L[l_off] and ``zbuf`` its inverted 32-blocks."""
    if len(panel) == 0:
        return
    rc = _lib.load().dpl_trsm_rb(uplo, n, L.data_ptr() + 8 * int(l_off), ldl, zbuf.data_ptr(), len(panel),
                                 panel.device(B.device).data_ptr(), B.data_ptr(), ldb, _lib.stream_ptr())
    _lib.check(rc, "trsm_rb")


# ----------------------------------------------------------------------------- TRSM
class _TrsmGroup:
    """Items sharing one triangle order: device items (gi = triangle index), triangle offsets, scratch."""

    def __init__(self, items, device, dtype, npos):
        tris = sorted({int(a) for a in items["a_off"]})
        idx = {a: i for i, a in enumerate(tris)}
        items = items.copy()
        items["gi"] = [idx[int(a)] for a in items["a_off"]]
        self.items = items
        self.max_m = int(items["m"].max())
        self.max_n = int(items["n"].max())
        self.ntri = len(tris)
        # pinned staging + asynchronous upload (kept alive with the group): building a group inside a
        # running program must not synchronise the stream
        dev = torch.device(device)
        hi = torch.from_numpy(items.view(np.uint8).copy())
        ht = torch.tensor(tris, dtype=torch.int64)
        if dev.type == "cuda":
            hi, ht = hi.pin_memory(), ht.pin_memory()
        self._host = (hi, ht)
        self.items_dev = hi.to(dev, non_blocking=True)
        self.tri_dev = ht.to(dev, non_blocking=True)
        nJ = (npos + 15) // 16
        self.work = torch.empty(self.ntri * nJ * 256, dtype=dtype, device=device)


def _trsm_groups(batch, side, B):
    key = (str(B.device), side, B.dtype)
    cache = getattr(batch, "_trsm_cache", None)
    if cache is None:
        cache = batch._trsm_cache = {}
    g = cache.get(key)
    if g is None:
        its = batch.items
        npos = its["m"] if side == dplasmaLeft else its["n"]
        g = [_TrsmGroup(its[npos == v], B.device, B.dtype, int(v)) for v in sorted(set(int(x) for x in npos))]
        cache[key] = g
    return g


TRSM_INVERSE_MIN_TILES = 8  # batches at least this large use inverse + MFMA GEMM


def _use_inverse(batch, side, B) -> bool:
    import os
    thr = int(os.environ.get("DPLASMA_TRSM_INVERSE_MIN_TILES", TRSM_INVERSE_MIN_TILES))
    if thr <= 0 or len(batch) < thr or B.dtype not in (torch.float64, torch.float32, torch.complex128,
                                                       torch.complex64):
        return False
    tris = set(int(a) for a in batch.items["a_off"])
    return len(tris) == 1


_IDENT = {}


def _identity(n, dtype, device):
    key = (n, dtype, str(device))
    t = _IDENT.get(key)
    if t is None:
        t = torch.eye(n, dtype=dtype, device=device).t().contiguous().view(-1)  # column-major
        _IDENT[key] = t
    return t


class _InvPlan:
    """Per-batch resources for TRSM = apply(op(T)^-1): inverse buffer, copy and GEMM batches."""

    def __init__(self, batch, side, B):
        its = batch.items
        npos = int(its["m"].max()) if side == dplasmaLeft else int(its["n"].max())
        self.n = npos
        self.inv = torch.empty(npos * npos, dtype=B.dtype, device=B.device)
        self.inv_batch = TileBatch().add(int(its["a_off"][0]), npos, npos, b_off=0).finalize()
        # scratch copy of B, one slot per item (ld = max rows)
        self.ld = int(its["m"].max())
        slot = self.ld * int(its["n"].max())
        self.scratch = torch.empty(max(1, len(its)) * slot, dtype=B.dtype, device=B.device)
        self.copy = TileBatch()
        self.gemm = GemmBatch()
        for j, it in enumerate(its):
            m, n = int(it["m"]), int(it["n"])
            self.copy.add(int(it["b_off"]), m, n, b_off=j * slot)
            if side == dplasmaLeft:   # B = Inv * S
                self.gemm.add(int(it["b_off"]), m, n, [(0, j * slot, m)])
            else:                     # B = S * Inv
                self.gemm.add(int(it["b_off"]), m, n, [(j * slot, 0, n)])
        self.copy.finalize()
        self.gemm.finalize()


def _trsm_via_inverse(side, uplo, trans, diag, alpha, A, lda, B, ldb, batch):
    plan = getattr(batch, "_inv_plan", None)
    if plan is None or plan.inv.device != B.device or plan.inv.dtype != B.dtype:
        plan = batch._inv_plan = _InvPlan(batch, side, B)
    n = plan.n
    inv2 = plan.inv
    inv2.copy_(_identity(n, B.dtype, B.device))
    # inv := op(T)^-1 by solving against the identity (strip kernel, n/16 workgroups)
    trsm_strip(side, uplo, trans, diag, 1.0, A, lda, inv2, n, plan.inv_batch)
    # scratch = B ; B = alpha * op-applied product
    geadd(0, dplasmaNoTrans, 1.0, B, ldb, 0.0, plan.scratch, plan.ld, plan.copy, copy=True)
    if side == dplasmaLeft:
        gemm(dplasmaNoTrans, dplasmaNoTrans, alpha, inv2, n, plan.scratch, plan.ld, 0.0, B, ldb, plan.gemm)
    else:
        gemm(dplasmaNoTrans, dplasmaNoTrans, alpha, plan.scratch, plan.ld, inv2, n, 0.0, B, ldb, plan.gemm)


def trsm_strip(side, uplo, trans, diag, alpha, A, lda, B, ldb, batch):
    """The strip kernel only (no inverse path)."""
    lib = _lib.load()
    batch.finalize()
    for sub in _trsm_groups(batch, side, B):
        sa = _lib.Scalar(alpha, B.dtype)
        rc = lib.dpl_trsm_batched(_lib.prec_code(B.dtype), side, uplo, trans, diag, len(sub.items),
                                  _pred_items(sub.items_dev).data_ptr(), sub.max_m, sub.max_n, sa.ptr, A.data_ptr(), lda,
                                  B.data_ptr(), ldb, sub.ntri, sub.tri_dev.data_ptr(), sub.work.data_ptr(),
                                  _lib.stream_ptr())
        _lib.check(rc, "trsm_batched")


def trsm(side: int, uplo: int, trans: int, diag: int, alpha, A: torch.Tensor, lda: int, B: torch.Tensor, ldb: int,
         batch: TileBatch):
    """For every item: solve op(T) X = alpha B (left) or X op(T) = alpha B (right) in place in B.

    item.a_off -> triangular tile in ``A``; item.b_off -> B tile; item m, n = B extent.
    """
    batch.finalize()
    if len(batch) == 0:
        return
    if _is_gpu(B):
        lib = _lib.load()
        if _use_inverse(batch, side, B):
            return _trsm_via_inverse(side, uplo, trans, diag, alpha, A, lda, B, ldb, batch)
        for sub in _trsm_groups(batch, side, B):
            sa = _lib.Scalar(alpha, B.dtype)
            rc = lib.dpl_trsm_batched(_lib.prec_code(B.dtype), side, uplo, trans, diag, len(sub.items),
                                      _pred_items(sub.items_dev).data_ptr(), sub.max_m, sub.max_n, sa.ptr, A.data_ptr(), lda,
                                      B.data_ptr(), ldb, sub.ntri, sub.tri_dev.data_ptr(), sub.work.data_ptr(),
                                      _lib.stream_ptr())
            _lib.check(rc, "trsm_batched")
        return
    left = side == dplasmaLeft
    for it in batch.items:
        m, n = int(it["m"]), int(it["n"])
        k = m if left else n
        t = _view(A, it["a_off"], k, k, lda)
        t = t.tril() if uplo == dplasmaLower else t.triu()
        if diag == dplasmaUnit:
            t = t - torch.diag_embed(torch.diagonal(t)) + torch.eye(k, dtype=t.dtype)
        opt = _op(t, trans)
        upper = (uplo == dplasmaUpper) != (trans != dplasmaNoTrans)
        b = _view(B, it["b_off"], m, n, ldb)
        x = torch.linalg.solve_triangular(opt, alpha * b, upper=upper, left=left)
        b.copy_(x)


# ----------------------------------------------------------------------------- generators
GEN_KIND = {"rnt": 0, "ghe": 1, "gsy": 2}


def generate(kind: str, A: torch.Tensor, lda: int, batch: TileBatch, gM: int, seed: int, bump=0.0):
    """Fill tiles with plrnt / plghe / plgsy values (bit-identical CPU/GPU)."""
    batch.finalize()
    if len(batch) == 0:
        return
    if _is_gpu(A):
        lib = _lib.load()
        items = batch.device_array(A.device)
        sb = _lib.Scalar(bump, A.dtype)
        rc = lib.dpl_generate(_lib.prec_code(A.dtype), GEN_KIND[kind], len(batch.items), items.data_ptr(),
                              batch.max_m, batch.max_n, A.data_ptr(), lda, int(gM), int(seed) & (2**64 - 1),
                              sb.ptr, _lib.stream_ptr())
        _lib.check(rc, "generate")
        return
    cplx = A.is_complex()
    for it in batch.items:
        m, n = int(it["m"]), int(it["n"])
        blk = lcg.generate_block(kind, int(it["gi"]), int(it["gj"]), m, n, gM, seed, cplx, bump)
        _view(A, it["a_off"], m, n, lda).copy_(torch.from_numpy(np.ascontiguousarray(blk)).to(A.dtype))


# ----------------------------------------------------------------------------- maps
# element selections (global coordinates); the kernels take the same codes
PART_FULL, PART_LOWER, PART_UPPER, PART_SLOWER, PART_SUPPER, PART_DIAG = 0, 1, 2, 3, 4, 5
_PART = {0: 0, 1: 1, 2: 2, 3: 3, 4: 4, 5: 5, dplasmaLower: 1, dplasmaUpper: 2, 123: 0}


def _part_mask(it, m, n, part):
    I = torch.arange(m).view(-1, 1) + int(it["gi"])
    J = torch.arange(n).view(1, -1) + int(it["gj"])
    if part == 1:
        return I >= J
    if part == 2:
        return I <= J
    if part == 3:
        return I > J
    if part == 4:
        return I < J
    if part == 5:
        return I == J
    return torch.ones(m, n, dtype=torch.bool)


def laset(uplo: int, alpha, beta, A: torch.Tensor, lda: int, batch: TileBatch):
    """Off-diagonal (global) entries := alpha, diagonal := beta, on the uplo part."""
    batch.finalize()
    if len(batch) == 0:
        return
    part = _PART.get(uplo, 0)
    if _is_gpu(A):
        sa, sb = _lib.Scalar(alpha, A.dtype), _lib.Scalar(beta, A.dtype)
        rc = _lib.load().dpl_laset(_lib.prec_code(A.dtype), part, len(batch.items),
                                   batch.device_array(A.device).data_ptr(), batch.max_m, batch.max_n, sa.ptr, sb.ptr,
                                   A.data_ptr(), lda, _lib.stream_ptr())
        _lib.check(rc, "laset")
        return
    for it in batch.items:
        m, n = int(it["m"]), int(it["n"])
        v = _view(A, it["a_off"], m, n, lda)
        I = torch.arange(m).view(-1, 1) + int(it["gi"])
        J = torch.arange(n).view(1, -1) + int(it["gj"])
        val = torch.where(I == J, torch.tensor(beta, dtype=A.dtype), torch.tensor(alpha, dtype=A.dtype))
        v.copy_(torch.where(_part_mask(it, m, n, part), val, v))


def geadd(uplo: int, trans: int, alpha, A: torch.Tensor, lda: int, beta, B: torch.Tensor, ldb: int,
          batch: TileBatch, copy: bool = False):
    """B = alpha*op(A) + beta*B (or B = op(A) when copy) on the uplo part; item a_off/b_off per tile."""
    batch.finalize()
    if len(batch) == 0:
        return
    part = _PART.get(uplo, 0)
    if _is_gpu(B):
        sa, sb = _lib.Scalar(alpha, B.dtype), _lib.Scalar(beta, B.dtype)
        rc = _lib.load().dpl_geadd(_lib.prec_code(B.dtype), part, trans, len(batch.items),
                                   batch.device_array(B.device).data_ptr(), batch.max_m, batch.max_n, sa.ptr,
                                   A.data_ptr(), lda, sb.ptr, B.data_ptr(), ldb, int(copy), _lib.stream_ptr())
        _lib.check(rc, "geadd")
        return
    for it in batch.items:
        m, n = int(it["m"]), int(it["n"])
        a = _view(A, it["a_off"], m, n, lda) if trans == dplasmaNoTrans else _op(_view(A, it["a_off"], n, m, lda), trans)
        b = _view(B, it["b_off"], m, n, ldb)
        new = a.clone() if copy else (alpha * a + (beta * b if beta != 0 else 0))
        b.copy_(torch.where(_part_mask(it, m, n, part), new, b))


def swap_transpose(A: torch.Tensor, ld: int, batch: TileBatch, conj: bool = False):
    """Per item: tile a (m x n at a_off) <- op(tile b)^T and tile b (n x m at b_off) <- op(tile a)^T,
    op = conj if ``conj``; a_off == b_off transposes a square tile in place (csrc/kernels/aux.hip)."""
    batch.finalize()
    if len(batch) == 0:
        return
    if _is_gpu(A):
        rc = _lib.load().dpl_swap_transpose(_lib.prec_code(A.dtype), len(batch.items),
                                            batch.device_array(A.device).data_ptr(), batch.max_m, batch.max_n,
                                            A.data_ptr(), ld, int(conj), _lib.stream_ptr())
        _lib.check(rc, "swap_transpose")
        return
    for it in batch.items:
        m, n = int(it["m"]), int(it["n"])
        a = _view(A, it["a_off"], m, n, ld)
        b = _view(A, it["b_off"], n, m, ld)
        na, nb = b.t().clone(), a.t().clone()
        if conj:
            na, nb = na.conj(), nb.conj()
        a.copy_(na)
        if int(it["a_off"]) != int(it["b_off"]):
            b.copy_(nb)


def copy_transpose(X: torch.Tensor, ldx: int, Y: torch.Tensor, ldy: int, batch: TileBatch, conj: bool = False,
                   upper_only: bool = False):
    """Per item: tile y (n x m at b_off in Y) <- op(tile x)^T (x: m x n at a_off in X), op = conj if
    ``conj``; ``upper_only`` leaves y's strictly lower part alone (csrc/kernels/aux.hip)."""
    batch.finalize()
    if len(batch) == 0:
        return
    if _is_gpu(Y):
        rc = _lib.load().dpl_copy_transpose(_lib.prec_code(Y.dtype), len(batch.items),
                                            batch.device_array(Y.device).data_ptr(), batch.max_m, batch.max_n,
                                            X.data_ptr(), ldx, Y.data_ptr(), ldy, int(conj), int(upper_only),
                                            _lib.stream_ptr())
        _lib.check(rc, "copy_transpose")
        return
    for it in batch.items:
        m, n = int(it["m"]), int(it["n"])
        x = _view(X, it["a_off"], m, n, ldx).t()
        if conj:
            x = x.conj()
        y = _view(Y, it["b_off"], n, m, ldy)
        if upper_only:
            y.copy_(torch.where(torch.ones(n, m, dtype=torch.bool, device=y.device).triu(), x, y))
        else:
            y.copy_(x)


def lascal(uplo: int, alpha, A: torch.Tensor, lda: int, batch: TileBatch):
    batch.finalize()
    if len(batch) == 0:
        return
    part = _PART.get(uplo, 0)
    if _is_gpu(A):
        sa = _lib.Scalar(alpha, A.dtype)
        rc = _lib.load().dpl_lascal(_lib.prec_code(A.dtype), part, len(batch.items),
                                    batch.device_array(A.device).data_ptr(), batch.max_m, batch.max_n, sa.ptr,
                                    A.data_ptr(), lda, _lib.stream_ptr())
        _lib.check(rc, "lascal")
        return
    for it in batch.items:
        m, n = int(it["m"]), int(it["n"])
        a = _view(A, it["a_off"], m, n, lda)
        a.copy_(torch.where(_part_mask(it, m, n, part), alpha * a, a))


# ----------------------------------------------------------------------------- norms
NORM_MAX, NORM_COLSUM, NORM_ROWSUM, NORM_SSQ = 0, 1, 2, 3


def tile_norm(kind: int, uplo: int, unit: bool, A: torch.Tensor, lda: int, batch: TileBatch) -> torch.Tensor:
    """Per-tile norm partials (float64, on A's device).

    MAX -> (ntiles,); COLSUM -> (ntiles, max_n); ROWSUM -> (ntiles, max_m); SSQ -> (ntiles, 2) (scale, ssq).
    """
    batch.finalize()
    nt = len(batch)
    ostride = {NORM_MAX: 1, NORM_COLSUM: max(batch.max_n, 1), NORM_ROWSUM: max(batch.max_m, 1), NORM_SSQ: 2}[kind]
    out = torch.zeros(nt, ostride, dtype=torch.float64, device=A.device)
    if nt == 0:
        return out
    part = _PART.get(uplo, 0)
    if _is_gpu(A):
        rc = _lib.load().dpl_tile_norm(_lib.prec_code(A.dtype), kind, part, int(unit), nt,
                                       batch.device_array(A.device).data_ptr(), A.data_ptr(), lda, out.data_ptr(),
                                       ostride, _lib.stream_ptr())
        _lib.check(rc, "tile_norm")
        return out
    for i, it in enumerate(batch.items):
        m, n = int(it["m"]), int(it["n"])
        a = _view(A, it["a_off"], m, n, lda).abs().to(torch.float64)
        mk = _part_mask(it, m, n, part)
        a = torch.where(mk, a, torch.zeros((), dtype=torch.float64))
        if unit:
            I = torch.arange(m).view(-1, 1) + int(it["gi"])
            J = torch.arange(n).view(1, -1) + int(it["gj"])
            a = torch.where((I == J) & mk, torch.ones((), dtype=torch.float64), a)
        if kind == NORM_MAX:
            out[i, 0] = a.max() if a.numel() else 0
        elif kind == NORM_COLSUM:
            out[i, :n] = a.sum(0)
        elif kind == NORM_ROWSUM:
            out[i, :m] = a.sum(1)
        else:
            mx = a.max() if a.numel() else torch.tensor(0.0, dtype=torch.float64)
            out[i, 0] = mx
            out[i, 1] = ((a / mx) ** 2).sum() if mx > 0 else 0.0
    return out


# ----------------------------------------------------------------------------- composite tile ops
def trtri_tile(uplo: int, diag: int, A: torch.Tensor, off: int, n: int, lda: int):
    """In-place inverse of the uplo triangle of one tile (CORE_ztrtri)."""
    if n <= 0:
        return
    if not _is_gpu(A):
        t = _view(A, off, n, n, lda)
        tri = t.tril() if uplo == dplasmaLower else t.triu()
        if diag == dplasmaUnit:
            tri = tri - torch.diag_embed(torch.diagonal(tri)) + torch.eye(n, dtype=t.dtype)
        inv = torch.linalg.solve_triangular(tri, torch.eye(n, dtype=t.dtype), upper=(uplo == dplasmaUpper))
        keep = torch.ones(n, n, dtype=torch.bool)
        keep = keep.tril(-1 if diag == dplasmaUnit else 0) if uplo == dplasmaLower else keep.triu(
            1 if diag == dplasmaUnit else 0)
        t.copy_(torch.where(keep, inv, t))
        return
    scratch = torch.eye(n, dtype=A.dtype, device=A.device).t().contiguous().view(-1)
    tb = TileBatch().add(int(off), n, n, b_off=0).finalize()
    trsm_strip(dplasmaLeft, uplo, dplasmaNoTrans, diag, 1.0, A, lda, scratch, n, tb)
    part = (3 if diag == dplasmaUnit else 1) if uplo == dplasmaLower else (4 if diag == dplasmaUnit else 2)
    cb = TileBatch().add(0, n, n, b_off=int(off)).finalize()
    geadd(part, dplasmaNoTrans, 1.0, scratch, n, 0.0, A, lda, cb, copy=True)


def lauum_tile(uplo: int, A: torch.Tensor, off: int, n: int, lda: int):
    """In-place L^H L (lower) or U U^H (upper) of one tile (CORE_zlauum)."""
    if n <= 0:
        return
    T = torch.zeros(n * n, dtype=A.dtype, device=A.device)
    W = torch.zeros(n * n, dtype=A.dtype, device=A.device)
    part = 1 if uplo == dplasmaLower else 2
    cb = TileBatch().add(int(off), n, n, b_off=0).finalize()
    geadd(part, dplasmaNoTrans, 1.0, A, lda, 0.0, T, n, cb, copy=True)
    gb = GemmBatch().add(0, n, n, [(0, 0, n)], MASK_LOWER if uplo == dplasmaLower else MASK_UPPER).finalize()
    if uplo == dplasmaLower:
        gemm(dplasmaConjTrans, dplasmaNoTrans, 1.0, T, n, T, n, 0.0, W, n, gb)
    else:
        gemm(dplasmaNoTrans, dplasmaConjTrans, 1.0, T, n, T, n, 0.0, W, n, gb)
    back = TileBatch().add(0, n, n, b_off=int(off)).finalize()
    geadd(part, dplasmaNoTrans, 1.0, W, n, 0.0, A, lda, back, copy=True)


# ----------------------------------------------------------------------------- LU primitives
def getrf_panel(A: torch.Tensor, off: int, m: int, n: int, lda: int, ipiv: torch.Tensor, info: torch.Tensor,
                info_base: int, pivot: bool = True):
    """LU of an m x n column-major panel in place; ipiv (int32, >= min(m,n)) gets 0-based panel rows."""
    if m <= 0 or n <= 0:
        return
    if _is_gpu(A):
        rc = _lib.load().dpl_getrf_panel(_lib.prec_code(A.dtype), m, n, A.data_ptr(), int(off), lda,
                                         ipiv.data_ptr() if ipiv is not None else None, info.data_ptr(),
                                         int(info_base), int(pivot), _lib.stream_ptr())
        _lib.check(rc, "getrf_panel")
        return
    P = _view(A, off, m, n, lda)
    kmax = min(m, n)
    if pivot:
        LU, piv, inf = torch.linalg.lu_factor_ex(P.clone())
        P.copy_(LU)
        if ipiv is not None:
            ipiv[:kmax] = (piv[:kmax] - 1).to(torch.int32)
        bad = int(inf)
        if bad > 0 and int(info[0]) == 0:
            info[0] = info_base + bad
        return
    for j in range(kmax):
        d = P[j, j]
        if d == 0:
            if int(info[0]) == 0:
                info[0] = info_base + j + 1
            continue
        P[j + 1:, j] /= d
        if j + 1 < n:
            P[j + 1:, j + 1:] -= torch.outer(P[j + 1:, j], P[j, j + 1:])
    if ipiv is not None:
        ipiv[:kmax] = torch.arange(kmax, dtype=torch.int32)


ROW_PAIR = np.dtype([("dst", "<i8"), ("src", "<i8")])


def row_gather(dst: torch.Tensor, src: torch.Tensor, pairs: np.ndarray, ncols: int, ld_dst: int, ld_src: int,
               _cache={}):
    """dst row at pairs[i].dst := src row at pairs[i].src (ncols elements each, column strides ld_*)."""
    if len(pairs) == 0 or ncols <= 0:
        return
    if _is_gpu(dst):
        dev = torch.from_numpy(np.ascontiguousarray(pairs).view(np.uint8).copy()).to(dst.device, non_blocking=False)
        rc = _lib.load().dpl_row_gather(_lib.prec_code(dst.dtype), dst.data_ptr(), src.data_ptr(), dev.data_ptr(),
                                        len(pairs), ncols, ld_dst, ld_src, _lib.stream_ptr())
        _lib.check(rc, "row_gather")
        return
    for p in pairs:
        d = torch.as_strided(dst, (ncols,), (ld_dst,), int(p["dst"]))
        s = torch.as_strided(src, (ncols,), (ld_src,), int(p["src"]))
        d.copy_(s)


# ----------------------------------------------------------------------------- diagonal scaling (LDL^H)
def diag_scale(part: int, cols: bool, D: torch.Tensor, ldd: int, B: torch.Tensor, ldb: int, batch: TileBatch):
    """B_tile(i, j) /= d (d = D_tile(j, j) if cols else D_tile(i, i)) on the part mask; a_off -> D tile, b_off -> B tile."""
    batch.finalize()
    if len(batch) == 0:
        return
    p = _PART.get(part, 0)
    if _is_gpu(B):
        rc = _lib.load().dpl_diag_scale(_lib.prec_code(B.dtype), p, int(cols), len(batch.items),
                                        batch.device_array(B.device).data_ptr(), batch.max_m, batch.max_n,
                                        D.data_ptr(), ldd, B.data_ptr(), ldb, _lib.stream_ptr())
        _lib.check(rc, "diag_scale")
        return
    for it in batch.items:
        m, n = int(it["m"]), int(it["n"])
        b = _view(B, it["b_off"], m, n, ldb)
        k = n if cols else m
        d = torch.as_strided(D, (k,), (ldd + 1,), int(it["a_off"]))
        new = b / (d.view(1, -1) if cols else d.view(-1, 1))
        b.copy_(torch.where(_part_mask(it, m, n, p), new, b))


# ----------------------------------------------------------------------------- random butterflies
def butterfly(A, r: torch.Tensor, size: int, side: int, trans: int):
    """One butterfly level on a one-process descriptor, element-wise O(m n) (csrc/kernels/butterfly.hip):
    A := B A / B^T A (side Left) or A B / A B^T (Right), B block diagonal with blocks
    1/sqrt(2) [R0 R1; R0 -R1] of order ``size``, R the real vector ``r`` (length = the order)."""
    from ..descriptor import STORAGE_TILE
    left = side == dplasmaLeft
    m, n = A.m, A.n
    order = m if left else n
    if size < 2 or size % 2 or order % size:
        raise ValueError("butterfly: size must be even and divide the order")
    form = 0 if left == (trans == dplasmaNoTrans) else 1
    if _is_gpu(A.data):
        if A.storage == STORAGE_TILE:
            si, sj = A.mb * A.nb, A.llmt * A.mb * A.nb
        else:
            si, sj = A.mb, A.nb * A.ld
        base = A.offset(0, 0) if (A.mt and A.nt) else 0
        rd = r.to(device=A.data.device, dtype=torch.float64).contiguous()
        buf = A.data[base:]
        rc = _lib.load().dpl_butterfly(_lib.prec_code(A.dtype), side, trans, m, n, size, rd.data_ptr(), buf.data_ptr(),
                                       si, sj, A.mb, A.nb, A.ld, _lib.stream_ptr())
        _lib.check(rc, "butterfly")
        return
    D = A.to_dense_local()
    X = D if left else D.t()
    h = size // 2
    idx = torch.arange(order // 2)
    i0 = (idx // h) * size + idx % h
    i1 = i0 + h
    rr = r.to(torch.float64).cpu()
    s = 1.0 / math.sqrt(2.0)
    r0 = rr[i0].to(D.dtype).view(-1, 1)
    r1 = rr[i1].to(D.dtype).view(-1, 1)
    x0, x1 = X[i0].clone(), X[i1].clone()
    if form == 0:
        a, b = r0 * x0, r1 * x1
        X[i0], X[i1] = s * (a + b), s * (a - b)
    else:
        X[i0], X[i1] = s * r0 * (x0 + x1), s * r1 * (x0 - x1)
    A.from_dense(D)


# ----------------------------------------------------------------------------- device-pivoting LU
QR_PANEL_MAXW = 256   # widest panel of the single-launch Householder panel kernel (qr_panel.hip QP_R)


def _qp_pred(lib):
    """Hand the enclosing batch predicate (ops/batch.py predicated) to the next panel launch: a device-decided
    branch's panels then exit at once when the flag is 0, like its batched launches."""
    from . import batch as _b
    f = _b._PRED[0]
    if f is None or not f.is_cuda:
        return False
    lib.dpl_qr_panel_set_pred(ctypes.c_void_p(f.data_ptr()))
    return True


def qr_panel_max_rows(device) -> int:
    """Tallest panel the persistent QR panel kernel factors in one launch (one workgroup per CU)."""
    if torch.device(device).type == "cuda":
        return int(_lib.load().dpl_qr_panel_max_rows())
    return 1 << 62


def qr_panel_workspace(nc: int, kf: int, dtype: torch.dtype, device) -> torch.Tensor:
    """Scratch for qr_panel on panels of nc columns (kf reflectors): reduction partials + barrier."""
    dev = torch.device(device)
    if dev.type == "cuda":
        nbytes = int(_lib.load().dpl_qr_panel_ws_bytes(_lib.prec_code(dtype), int(nc), int(kf)))
        return torch.zeros(nbytes // 8 + 8, dtype=torch.float64, device=dev)
    return torch.zeros(8, dtype=torch.float64)


QP_ITEM = np.dtype([("P0", "<u8"), ("rstride", "<i8"), ("V", "<u8"), ("Tm", "<u8"), ("ws", "<u8"), ("cnt", "<u8"),
                    ("ldp", "<i4"), ("rbl", "<i4"), ("M", "<i4"), ("nc", "<i4"), ("kf", "<i4"), ("R", "<i4"),
                    ("ldv", "<i4"), ("ldt", "<i4"), ("G", "<i4"), ("wbase", "<i4")])


class QrPanelMulti:
    """Several independent Householder panel factorisations in ONE persistent launch (real precisions,
    GPU; csrc/kernels/qr_panel.hip k_qr_panel_multi): panel e = (P, poff, ldp, rbl, rstride, M, nc, kf,
    V, voff, ldv, Tm, toff, ldt) with the semantics of ``qr_panel``.  Built once (items uploaded to the
    device, per-panel workspaces and barrier counters allocated); ``run`` re-launches.  On the CPU (or
    for complex types, or more workgroups than CUs) the panels are factored one by one by qr_panel."""

    def __init__(self, panels, dtype, device):
        self.panels = list(panels)
        self.dtype, self.device = dtype, torch.device(device)
        self.multi = (self.device.type == "cuda" and dtype in (torch.float32, torch.float64) and len(self.panels) > 0)
        if not self.multi:
            self.ws = qr_panel_workspace(max(p[6] for p in self.panels) if self.panels else 1,
                                         max(p[7] for p in self.panels) if self.panels else 1, dtype, device)
            return
        lib = _lib.load()
        if int(lib.dpl_qr_panel_item_bytes()) != QP_ITEM.itemsize:
            raise RuntimeError("QrPanelMulti: QpItem layout mismatch")
        prec, es = _lib.prec_code(dtype), torch.empty(0, dtype=dtype).element_size()
        n = len(self.panels)
        Gs = [max(1, -(-p[5] // 256)) for p in self.panels]
        self.total = sum(Gs)
        ncu = torch.cuda.get_device_properties(self.device).multi_processor_count
        if self.total > ncu:
            raise ValueError(f"QrPanelMulti: {self.total} workgroups > {ncu} CUs (split the group)")
        sizes = [int(lib.dpl_qr_panel_multi_ws_bytes(prec, int(p[6]), int(p[7]), g)) for p, g in zip(self.panels, Gs)]
        offs = np.concatenate([[0], np.cumsum([(x + 255) // 256 * 256 for x in sizes])]).astype(np.int64)
        self.wsbuf = torch.zeros(int(offs[-1]) // 8 + 32, dtype=torch.float64, device=self.device)
        self.cnt = torch.zeros(n, dtype=torch.int32, device=self.device)
        it = np.zeros(n, dtype=QP_ITEM)
        wb = 0
        for e, ((P, poff, ldp, rbl, rstride, M, nc, kf, V, voff, ldv, Tm, toff, ldt), G) in enumerate(
                zip(self.panels, Gs)):
            if not 0 < rbl < M:
                rbl, rstride = 1 << 30, 0
                if ldp < M:
                    raise ValueError("QrPanelMulti: ldp < M")
            if not (0 < kf <= min(M, nc, 256)) or ldv < M or ldt < kf:
                raise ValueError("QrPanelMulti: bad panel shape")
            it[e] = (P.data_ptr() + poff * es, rstride, V.data_ptr() + voff * es, Tm.data_ptr() + toff * es,
                     self.wsbuf.data_ptr() + int(offs[e]), self.cnt.data_ptr() + 4 * e,
                     ldp, rbl, M, nc, kf, -(-M // G), ldv, ldt, G, wb)
            wb += G
        self.items = torch.from_numpy(it.view(np.uint8).copy()).to(self.device)

    def run(self, info: torch.Tensor):
        if not self.multi:
            for (P, poff, ldp, rbl, rstride, M, nc, kf, V, voff, ldv, Tm, toff, ldt) in self.panels:
                if self.device.type == "cuda":
                    qr_panel(P, ldp, M, nc, kf, V[voff:], ldv, Tm[toff:], ldt, self.ws, info, rbl=rbl,
                             rstride=rstride, poff=poff)
                    continue
                # CPU: qr_panel addresses V / Tm from their first element -- factor into scratch
                vt = torch.zeros(ldv * kf, dtype=V.dtype)
                tt = Tm[toff: toff + ldt * kf].clone()
                qr_panel(P, ldp, M, nc, kf, vt, ldv, tt, ldt, self.ws, info, rbl=rbl, rstride=rstride, poff=poff)
                V[voff: voff + ldv * kf] = vt
                Tm[toff: toff + ldt * kf] = tt
            return
        lib = _lib.load()
        pr = _qp_pred(lib)
        rc = lib.dpl_qr_panel_multi(_lib.prec_code(self.dtype), len(self.panels), self.total,
                                    self.items.data_ptr(), self.cnt.data_ptr(), info.data_ptr(), _lib.stream_ptr())
        if pr:
            lib.dpl_qr_panel_set_pred(ctypes.c_void_p(0))
        _lib.check(rc, "qr_panel_multi")


def _larft_cpu(V: torch.Tensor, tau: torch.Tensor) -> torch.Tensor:
    """Compact-WY T (upper triangular, dlarft forward/columnwise) of explicit reflectors V."""
    k = V.shape[1]
    T = torch.zeros(k, k, dtype=V.dtype)
    G = V.mH @ V
    for j in range(k):
        T[j, j] = tau[j]
        if j:
            T[:j, j] = -tau[j] * (T[:j, :j] @ G[:j, j])
    return T


def sum_partials(src: torch.Tensor, stride: int, S: int, L: int, dst: torch.Tensor):
    """dst[:L] = sum over s < S of src[s*stride : s*stride + L] (split-K partials)."""
    if _is_gpu(dst):
        rc = _lib.load().dpl_sum_partials(_lib.prec_code(dst.dtype), src.data_ptr(), int(stride), int(S), int(L),
                                          dst.data_ptr(), _lib.stream_ptr())
        _lib.check(rc, "sum_partials")
        return
    torch.sum(torch.as_strided(src, (S, L), (stride, 1), 0), 0, out=dst[:L])


def qr_panel(P: torch.Tensor, ldp: int, M: int, nc: int, kf: int, V: torch.Tensor, ldv: int, Tm: torch.Tensor,
             ldt: int, ws: torch.Tensor, info: torch.Tensor, rbl: int = 0, rstride: int = 0, poff: int = 0):
    """Householder QR of the column-major M x nc panel P (ld ldp), first kf columns (s/d/c/z).

    P := R (upper) + V (strictly lower) with the remaining nc - kf columns updated by Q^H;
    V := the kf reflectors explicitly (unit diagonal, zeros above); Tm(0:kf, 0:kf) := the
    compact-WY T (upper part; the strictly lower part is not written).  GPU: one persistent
    launch (csrc/kernels/qr_panel.hip); CPU: LAPACK geqrf through torch + dlarft.
    The panel starts at element poff of P; 0 < rbl < M: its rows come in blocks of rbl rows,
    rstride elements apart (a column of tiles in TILE storage, addressed in place, ldp = mb)."""
    if kf <= 0:
        return
    if _is_gpu(P):
        lib = _lib.load()
        pr = _qp_pred(lib)
        rc = lib.dpl_qr_panel(_lib.prec_code(P.dtype), P.data_ptr() + poff * P.element_size(), ldp, int(rbl),
                              int(rstride), M, nc, kf, V.data_ptr(), ldv, Tm.data_ptr(), ldt, ws.data_ptr(),
                              info.data_ptr(), _lib.stream_ptr())
        if pr:
            lib.dpl_qr_panel_set_pred(ctypes.c_void_p(0))   # (the library's other callers launch unpredicated)
        _lib.check(rc, "qr_panel")
        return
    if 0 < rbl < M or poff:
        if not 0 < rbl < M:
            rbl, rstride = M, 0
        blocks = [torch.as_strided(P, (min(rbl, M - r0), nc), (1, ldp), poff + (r0 // rbl) * rstride)
                  for r0 in range(0, M, rbl)]
        tmp = torch.cat(blocks, 0).T.contiguous().view(-1)   # column-major M x nc
        qr_panel(tmp, M, M, nc, kf, V, ldv, Tm, ldt, ws, info)
        res = torch.as_strided(tmp, (M, nc), (1, M), 0)
        r0 = 0
        for blk in blocks:
            blk.copy_(res[r0:r0 + blk.shape[0]])
            r0 += blk.shape[0]
        return
    A = torch.as_strided(P, (M, nc), (1, ldp), 0)
    a, tau = torch.geqrf(A[:, :kf].clone())
    Vx = torch.tril(a, -1) + torch.eye(M, kf, dtype=P.dtype)
    T = _larft_cpu(Vx, tau)
    if nc > kf:
        A[:, kf:] -= Vx @ (T.mH @ (Vx.mH @ A[:, kf:]))
    A[:, :kf] = a
    torch.as_strided(V, (M, kf), (1, ldv), 0).copy_(Vx)
    tv = torch.as_strided(Tm, (kf, kf), (1, ldt), 0)
    tv.copy_(torch.where(torch.ones(kf, kf, dtype=torch.bool).triu(), T, tv))


import os as _os
# base block width of the recursive panel LU (lu_piv.hip LU_MAXBW = 64); DPLASMA_LU_BW=32 selects the
# 64 KiB-LDS block kernel, which can share a CU with a trailing-update GEMM workgroup under look-ahead
LU_BW = int(_os.environ.get("DPLASMA_LU_BW", "64"))


def lu_workspace(m: int, device) -> torch.Tensor:
    """Scratch for lu_block / PanelLU on panels of up to m rows (pivot candidates, barrier data)."""
    dev = torch.device(device)
    if dev.type == "cuda":
        nbytes = int(_lib.load().dpl_lu_block_ws_bytes(int(m)))
        return torch.zeros(nbytes // 8 + 8, dtype=torch.float64, device=dev)
    return torch.zeros(8, dtype=torch.float64)


def lu_block(P: torch.Tensor, ld: int, m: int, c0: int, cend: int, ipiv: torch.Tensor, ws: torch.Tensor,
             cnt: torch.Tensor, info: torch.Tensor, info_base: int, pivot: bool = True):
    """Unblocked LU with partial pivoting of panel columns [c0, cend), rows [c0, m) of the column-major
    buffer P (ld): swaps only inside the block columns, ipiv[j] = panel-relative pivot row."""
    if cend <= c0 or m <= c0:
        return
    if _is_gpu(P):
        rc = _lib.load().dpl_lu_block(_lib.prec_code(P.dtype), P.data_ptr(), ld, m, c0, cend, ipiv.data_ptr(),
                                      ws.data_ptr(), cnt.data_ptr(), info.data_ptr(), int(info_base), int(pivot),
                                      _lib.stream_ptr())
        _lib.check(rc, "lu_block")
        return
    A = torch.as_strided(P, (m, cend), (1, ld), 0)
    for j in range(c0, min(cend, m)):
        col = A[j:, j]
        p = j + int(torch.argmax(col.abs() if not col.is_complex() else col.real.abs() + col.imag.abs())) \
            if pivot else j
        ipiv[j] = p
        if p != j:
            t = A[j, c0:cend].clone()
            A[j, c0:cend] = A[p, c0:cend]
            A[p, c0:cend] = t
        d = A[j, j]
        if d == 0:
            if int(info[0]) == 0:
                info[0] = info_base + j + 1
        else:
            A[j + 1:, j] /= d
        if j + 1 < cend:
            A[j + 1:, j + 1:cend] -= torch.outer(A[j + 1:, j], A[j, j + 1:cend])


BAD_PIVOT = -1001   # info code of an out-of-range pivot (csrc/kernels/lu_piv.hip report_bad_pivot)


def _bad_pivot(info):
    """Record BAD_PIVOT in info over 0 or a positive singular-column index (never over another failure)."""
    if info is not None and int(info[0]) >= 0:
        info[0] = BAD_PIVOT


def _iptr(t):
    return t.data_ptr() if t is not None else None


def laswp_panel(P: torch.Tensor, ld: int, ca: int, cb: int, ipiv: torch.Tensor, i0: int, i1: int, m: int = None,
                info: torch.Tensor = None):
    """Sequential row interchanges i <-> ipiv[i] (i in [i0, i1)) on columns [ca, cb) of panel P (m rows).
    A pivot outside [i, m) moves nothing and sets info to BAD_PIVOT."""
    if cb <= ca or i1 <= i0:
        return
    m = (1 << 31) - 1 if m is None else int(m)
    if _is_gpu(P):
        rc = _lib.load().dpl_laswp_panel(_lib.prec_code(P.dtype), P.data_ptr(), ld, m, ca, cb, ipiv.data_ptr(), i0, i1,
                                         _iptr(info), _lib.stream_ptr())
        _lib.check(rc, "laswp_panel")
        return
    pv = [int(x) for x in ipiv[i0:i1]]
    if any(p < i0 + q or p >= m for q, p in enumerate(pv)):
        _bad_pivot(info)
        return
    nrow = max(pv) + 1
    A = torch.as_strided(P, (max(nrow, i1), cb - ca), (1, ld), ca * ld)
    for i in range(i0, i1):
        p = int(ipiv[i])
        if p != i:
            t = A[i].clone()
            A[i] = A[p]
            A[p] = t


def piv_moves(ipiv: torch.Tensor, kb: int, dst: torch.Tensor, src: torch.Tensor, cnt: torch.Tensor, mrel: int = None,
              info: torch.Tensor = None):
    """Net row moves of the sequential interchanges ipiv[:kb]: row dst[t] receives former row src[t].
    Pivots must lie in [i, mrel); otherwise no moves (cnt = 0) and info = BAD_PIVOT."""
    mrel = (1 << 31) - 1 if mrel is None else int(mrel)
    if _is_gpu(ipiv):
        rc = _lib.load().dpl_piv_moves(ipiv.data_ptr(), kb, mrel, dst.data_ptr(), src.data_ptr(), cnt.data_ptr(),
                                       _iptr(info), _lib.stream_ptr())
        _lib.check(rc, "piv_moves")
        return
    if any(int(ipiv[i]) < i or int(ipiv[i]) >= mrel for i in range(kb)):
        cnt[0] = 0
        _bad_pivot(info)
        return
    cur = {}
    for i in range(kb):
        p = int(ipiv[i])
        if p != i:
            a, b = cur.get(i, i), cur.get(p, p)
            cur[i], cur[p] = b, a
    moves = sorted((d, s_) for d, s_ in cur.items() if d != s_)
    for t, (d, s_) in enumerate(moves):
        dst[t] = d
        src[t] = s_
    cnt[0] = len(moves)


def rows_perm_col(A: torch.Tensor, ld: int, mb: int, rowoff: torch.Tensor, coff: int, ncols: int, src: torch.Tensor,
                  r0: int, cnt: int, buf: torch.Tensor, info: torch.Tensor = None):
    """One tile column's rows [r0, r0 + cnt) take the former rows src[0:cnt) (element (r, c) at
    rowoff[r // mb] + r % mb + coff + c * ld): the deferred left interchanges of getrf_1d.  buf: cnt x ncols scratch."""
    if cnt <= 0 or ncols <= 0:
        return
    if _is_gpu(A):
        rc = _lib.load().dpl_rows_perm_col(_lib.prec_code(A.dtype), A.data_ptr(), ld, mb, rowoff.data_ptr(),
                                           int(rowoff.numel()), int(coff), int(ncols), src.data_ptr(), int(r0), int(cnt),
                                           buf.data_ptr(), _iptr(info), _lib.stream_ptr())
        _lib.check(rc, "rows_perm_col")
        return
    ro = rowoff.to(torch.int64)
    cols = torch.arange(ncols, dtype=torch.int64) * ld + int(coff)

    def addr(rows):
        rows = rows.to(torch.int64)
        return (ro[rows // mb] + rows % mb)[:, None] + cols[None, :]
    vals = A[addr(src[:cnt])].clone()
    A[addr(torch.arange(r0, r0 + cnt))] = vals


def rows_permute(A: torch.Tensor, ld: int, mb: int, r0: int, rowoff: torch.Tensor, coloff: torch.Tensor,
                 ncols: torch.Tensor, nb: int, dst: torch.Tensor, src: torch.Tensor, cnt: torch.Tensor, maxcnt: int,
                 info: torch.Tensor = None):
    """In place, one process: A[r0 + dst[t], col c] := old A[r0 + src[t], col c] on the flattened local
    tile columns (coloff[j], ncols[j]) -- rows_move gather + scatter without the staging buffer."""
    nct = int(coloff.numel())
    if nct == 0:
        return
    if _is_gpu(A):
        rc = _lib.load().dpl_rows_permute(_lib.prec_code(A.dtype), A.data_ptr(), ld, mb, r0, rowoff.data_ptr(),
                                          int(rowoff.numel()), coloff.data_ptr(), ncols.data_ptr(), nct, nb,
                                          dst.data_ptr(), src.data_ptr(), cnt.data_ptr(), maxcnt, _iptr(info),
                                          _lib.stream_ptr())
        _lib.check(rc, "rows_permute")
        return
    n = int(cnt[0])
    R = [r0 + int(x) for x in list(src[:n]) + list(dst[:n])]
    if any(r < 0 or r // mb >= rowoff.numel() or int(rowoff[r // mb]) < 0 for r in R):
        _bad_pivot(info)   # a corrupt move list: nothing moves (as the kernel)
        return
    buf = torch.zeros(maxcnt * nct * nb, dtype=A.dtype, device=A.device)
    rows_move(True, A, ld, mb, r0, rowoff, coloff, ncols, nb, src, cnt, maxcnt, buf, maxcnt, info)
    rows_move(False, A, ld, mb, r0, rowoff, coloff, ncols, nb, dst, cnt, maxcnt, buf, maxcnt, info)


def rows_xord(dst: torch.Tensor, src: torch.Tensor, cnt: torch.Tensor, r0: int, mb: int, prow: torch.Tensor, me: int,
              P: int, ldx: int, xo: torch.Tensor, info: torch.Tensor = None):
    """Classify the net moves (dst[t] <- src[t], rows r0 + ...) for the point-to-point exchange between process rows
    (the reference's SWAP_COLLECT / SWAP_SND, src/zgetrf_ptgpanel.jdf:825-984): xo[t] = 1<<30 | q<<16 | ord when my
    staged source row goes to process row q, 1<<29 | q<<16 | ord when it arrives from q, -1 otherwise; ord is the
    move's rank inside its (source row, destination row) class -- the same on both sides.  prow[view tile row] =
    its process row."""
    if _is_gpu(dst):
        rc = _lib.load().dpl_rows_xord(dst.data_ptr(), src.data_ptr(), cnt.data_ptr(), r0, mb, prow.data_ptr(),
                                       int(prow.numel()), me, P, ldx, xo.data_ptr(), _iptr(info), _lib.stream_ptr())
        _lib.check(rc, "rows_xord")
        return
    n = int(cnt[0])
    nrt = int(prow.numel())
    nxt = {}
    xo.fill_(-1)
    for t in range(n):
        Rs, Rd = r0 + int(src[t]), r0 + int(dst[t])
        if not (0 <= Rs and 0 <= Rd and Rs // mb < nrt and Rd // mb < nrt):
            _bad_pivot(info)
            continue
        so, dd = int(prow[Rs // mb]), int(prow[Rd // mb])
        if so == dd or (so != me and dd != me):
            continue
        key = (so, dd)
        o = nxt.get(key, 0)
        nxt[key] = o + 1
        if o >= ldx:
            _bad_pivot(info)
            continue
        xo[t] = ((1 << 30) | (dd << 16) | o) if so == me else ((1 << 29) | (so << 16) | o)


def rows_xcopy(pack: bool, tmp: torch.Tensor, ldb: int, W: int, xo: torch.Tensor, cnt: torch.Tensor, maxcnt: int,
               bufs, ldx: int):
    """pack: bufs[q][ord + c ldx] = tmp[t + c ldb] for my moves leaving for process row q; unpack: the reverse for
    the moves arriving from q (c < W).  bufs: a device int64 tensor of buffer addresses (GPU) or a list of tensors
    indexed by process row (CPU)."""
    if W <= 0 or maxcnt <= 0:
        return
    if _is_gpu(tmp):
        rc = _lib.load().dpl_rows_xcopy(_lib.prec_code(tmp.dtype), int(pack), tmp.data_ptr(), ldb, W, xo.data_ptr(),
                                        cnt.data_ptr(), maxcnt, bufs.data_ptr(), ldx, _lib.stream_ptr())
        _lib.check(rc, "rows_xcopy")
        return
    n = int(cnt[0])
    bit = 30 if pack else 29
    for t in range(n):
        x = int(xo[t])
        if x < 0 or not (x >> bit) & 1:
            continue
        q, o = (x >> 16) & 0x1FFF, x & 0xFFFF
        tv = torch.as_strided(tmp, (W,), (ldb,), t)
        bv = torch.as_strided(bufs[q], (W,), (ldx,), o)
        if pack:
            bv.copy_(tv)
        else:
            tv.copy_(bv)


def rows_move(gather: bool, A: torch.Tensor, ld: int, mb: int, r0: int, rowoff: torch.Tensor, coloff: torch.Tensor,
              ncols: torch.Tensor, nb: int, rows: torch.Tensor, cnt: torch.Tensor, maxcnt: int, buf: torch.Tensor,
              ldb: int, info: torch.Tensor = None):
    """gather: buf[t, c] = A[r0 + rows[t], col c] (0 where the row is not local);
    scatter: A[r0 + rows[t], col c] = buf[t, c] where local.  Columns: the flattened local tile
    columns (coloff[j], ncols[j]); buf is column-major with leading dimension ldb."""
    nct = int(coloff.numel())
    if nct == 0:
        return
    if _is_gpu(A):
        rc = _lib.load().dpl_rows_move(_lib.prec_code(A.dtype), int(gather), A.data_ptr(), ld, mb, r0,
                                       rowoff.data_ptr(), int(rowoff.numel()), coloff.data_ptr(), ncols.data_ptr(),
                                       nct, nb, rows.data_ptr(), cnt.data_ptr(), maxcnt, buf.data_ptr(), ldb,
                                       _iptr(info), _lib.stream_ptr())
        _lib.check(rc, "rows_move")
        return
    n = int(cnt[0])
    for t in range(n):
        R = r0 + int(rows[t])
        inview = 0 <= R and R // mb < rowoff.numel()
        if not inview:   # a corrupt move list: reported, never dereferenced
            _bad_pivot(info)
        ro = int(rowoff[R // mb]) if inview else -1
        for j in range(nct):
            w = int(ncols[j])
            if w == 0:
                continue
            bv = torch.as_strided(buf, (w,), (ldb,), j * nb * ldb + t)
            if ro < 0:
                if gather:
                    bv.zero_()
                continue
            av = torch.as_strided(A, (w,), (ld,), ro + R % mb + int(coloff[j]))
            if gather:
                bv.copy_(av)
            else:
                av.copy_(bv)


class PanelLU:
    """Recursive LU with partial pivoting of one tall column-major panel (m x n, ld), device-resident:
    halves until <= LU_BW columns (lu_block), then laswp + TRSM + MFMA GEMM to join the halves
    (the dgetrf2 recursion; reference CORE_zgetrf_rectil's role).  The TRSM / GEMM batches of
    every recursion node are built once here and re-used by every run."""

    def __init__(self, buf: torch.Tensor, ld: int, m: int, n: int, pivot: bool = True, bw: int = None):
        self.buf, self.ld, self.m, self.n, self.pivot = buf, ld, m, n, pivot
        # base block width: <= 32 columns select the 64 KiB LDS block kernel, which leaves room on a CU for a
        # trailing-update GEMM workgroup beside it (callers that overlap the panel with updates)
        self.bw = int(bw) if bw else LU_BW
        self.plan = []
        kf = min(m, n)
        self._rec(0, kf)
        if n > kf:   # wide panel: the columns past the last row only get the swaps and U = L^-1 A
            self.plan.append(("laswp", kf, n, 0, kf))
            self.plan.append(("trsm", TileBatch().add(0, kf, n - kf, b_off=kf * ld).finalize()))

    def _rec(self, c0: int, n: int):
        ld, m = self.ld, self.m
        if n <= self.bw:
            self.plan.append(("block", c0, c0 + n))
            return
        n1 = (n // 2 + 15) // 16 * 16
        self._rec(c0, n1)
        c1 = c0 + n1
        self.plan.append(("laswp", c1, c0 + n, c0, c1))
        tb = TileBatch().add(c0 + c0 * ld, n1, n - n1, b_off=c0 + c1 * ld).finalize()
        self.plan.append(("trsm", tb))
        if m > c1:
            gb = GemmBatch().add(c1 + c1 * ld, m - c1, n - n1, [(c1 + c0 * ld, c0 + c1 * ld, n1)]).finalize()
            self.plan.append(("gemm", gb))
        self._rec(c1, n - n1)
        self.plan.append(("laswp", c0, c1, c1, c0 + n))

    def run(self, ipiv: torch.Tensor, ws: torch.Tensor, cnt: torch.Tensor, info: torch.Tensor, info_base: int):
        P, ld, m = self.buf, self.ld, self.m
        for op in self.plan:
            if op[0] == "block":
                lu_block(P, ld, m, op[1], op[2], ipiv, ws, cnt, info, info_base, self.pivot)
            elif op[0] == "laswp":
                if self.pivot:
                    laswp_panel(P, ld, op[1], op[2], ipiv, op[3], op[4], m=m, info=info)
            elif op[0] == "trsm":
                trsm(dplasmaLeft, dplasmaLower, dplasmaNoTrans, dplasmaUnit, 1.0, P, ld, P, ld, op[1])
            else:
                gemm(dplasmaNoTrans, dplasmaNoTrans, -1.0, P, ld, P, ld, 1.0, P, ld, op[1])
