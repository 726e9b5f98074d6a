"""Item batches: the unit of work handed to one batched kernel launch.

A batch is built once (host numpy records, ``ENQ`` phase) and uploaded once
per device; executing it is a single kernel launch on GPU, or a loop of
PyTorch tile operations on the CPU reference path.  The record layouts match
``csrc/kernels/common.h`` / ``gemm.hip`` exactly.
"""
from __future__ import annotations

import contextlib

import numpy as np
import torch

GEMM_ITEM = np.dtype([("c_off", "<i8"), ("kt_beg", "<i4"), ("kt_cnt", "<i4"), ("m", "<i4"), ("n", "<i4"),
                      ("flags", "<i4"), ("pad", "<i4")])
KPAIR = np.dtype([("a_off", "<i8"), ("b_off", "<i8"), ("k", "<i4"), ("pad", "<i4")])
TILE_ITEM = np.dtype([("a_off", "<i8"), ("b_off", "<i8"), ("m", "<i4"), ("n", "<i4"), ("gi", "<i4"), ("gj", "<i4")])
assert GEMM_ITEM.itemsize == 32 and KPAIR.itemsize == 24 and TILE_ITEM.itemsize == 32

MASK_FULL, MASK_LOWER, MASK_UPPER = 0, 1, 2

# Predicated issue (models/lu_qr.py's device-decided steps): while a device flag is set, every batch handed to a
# kernel is a copy whose item sizes (m, n: int32 words 4 and 5 of both 32-byte records) are multiplied by the
# flag on the device -- flag 0 turns every launch of the branch into workgroups that exit at once, without the
# host ever reading the flag.  Nested predicates multiply.
_PRED = [None]


@contextlib.contextmanager
def predicated(flag):
    """Issue the enclosed batch launches under a device int32 flag (shape [1]): 1 runs them, 0 skips them."""
    old = _PRED[0]
    _PRED[0] = flag if old is None else old * flag
    try:
        yield
    finally:
        _PRED[0] = old


@contextlib.contextmanager
def unpredicated():
    """Launches that must run whatever the enclosing predicate (e.g. work whose result only feeds predicated
    launches, and which must not see skipped inputs)."""
    old = _PRED[0]
    _PRED[0] = None
    try:
        yield
    finally:
        _PRED[0] = old


def _pred(t: torch.Tensor) -> torch.Tensor:
    f = _PRED[0]
    if f is None or t.numel() == 0:
        return t
    p = t.clone()
    v = p.view(torch.int32).view(-1, 8)
    v[:, 4:6] *= f.to(device=p.device, dtype=torch.int32)
    return p


class _Uploadable:
    def __init__(self):
        self._dev = {}
        self._host = {}

    def _upload(self, arr: np.ndarray, device: torch.device) -> torch.Tensor:
        key = (id(arr), str(device))
        t = self._dev.get(key)
        if t is None:
            host = torch.from_numpy(arr.view(np.uint8).copy())
            if device.type == "cuda":
                host = host.pin_memory()
                t = host.to(device, non_blocking=True)
                # keep the pinned staging buffer for the batch's lifetime: the
                # async H2D copy must never read a recycled host block
                self._host[key] = host
            else:
                t = host
            self._dev[key] = t
        return t


class GemmBatch(_Uploadable):
    """C_i = beta*C_i + alpha * sum_j opA(A_ij) opB(B_ij) over a list of C tiles."""

    def __init__(self):
        super().__init__()
        self._items = []
        self._kps = []
        self.items = None
        self.kpairs = None
        self.max_m = self.max_n = 0
        self.vec_ok = True
        self.full = True   # every item whole 128x128 sub-tiles, every k-run a multiple of 16
        self._align = 0    # OR of all element offsets (vector-alignment test per dtype)
        self.flops_mnk = 0.0

    def add(self, c_off: int, m: int, n: int, kpairs, mask: int = MASK_FULL):
        """kpairs: iterable of (a_off, b_off, k)."""
        kp = list(kpairs)
        beg = len(self._kps)
        for (a, b, k) in kp:
            self._kps.append((a, b, k, 0))
            if a % 2 or b % 2:
                self.vec_ok = False
            self._align |= int(a) | int(b)
            if k % 16:
                self.full = False
            self.flops_mnk += float(m) * n * k
        if m % 128 or n % 128:
            self.full = False
        self._items.append((c_off, beg, len(kp), m, n, mask, 0))
        if c_off % 2:
            self.vec_ok = False
        self._align |= int(c_off)
        self.max_m = max(self.max_m, m)
        self.max_n = max(self.max_n, n)
        return self

    def add_arrays(self, c_off, m, n, kt_cnt, a_off, b_off, k, mask: int = MASK_FULL):
        """Vectorised add: items (c_off[i], m[i], n[i]) with kt_cnt[i] consecutive K-pairs taken from
        (a_off, b_off, k) in item order -- one numpy pass for millions of items."""
        c_off, m, n, kt_cnt = (np.asarray(x, dtype=np.int64).ravel() for x in (c_off, m, n, kt_cnt))
        a_off, b_off, k = (np.asarray(x, dtype=np.int64).ravel() for x in (a_off, b_off, k))
        ni = len(c_off)
        if ni == 0:
            return self
        m, n, kt_cnt = (np.broadcast_to(x, (ni,)) for x in (m, n, kt_cnt))
        nk = int(kt_cnt.sum())
        k = np.broadcast_to(k, (nk,))
        beg = len(self._kps) + sum(len(c) for c in getattr(self, "_kp_chunks", [])) + np.concatenate(
            [[0], np.cumsum(kt_cnt)[:-1]])
        items = np.zeros(ni, dtype=GEMM_ITEM)
        items["c_off"], items["kt_beg"], items["kt_cnt"] = c_off, beg, kt_cnt
        items["m"], items["n"], items["flags"] = m, n, mask
        kps = np.zeros(nk, dtype=KPAIR)
        kps["a_off"], kps["b_off"], kps["k"] = a_off, b_off, k
        if not hasattr(self, "_item_chunks"):
            self._item_chunks, self._kp_chunks = [], []
        self._item_chunks.append(items)
        self._kp_chunks.append(kps)
        if (a_off % 2).any() or (b_off % 2).any() or (c_off % 2).any():
            self.vec_ok = False
        self._align |= int(np.bitwise_or.reduce(np.concatenate([a_off, b_off, c_off])))
        if (k % 16).any() or (m % 128).any() or (n % 128).any():
            self.full = False
        # flops: sum over items of m*n*sum(k of its pairs)
        ksum = np.add.reduceat(k, np.concatenate([[0], np.cumsum(kt_cnt)[:-1]])) if nk else np.zeros(ni)
        self.flops_mnk += float((m.astype(np.float64) * n * ksum).sum())
        self.max_m = max(self.max_m, int(m.max()))
        self.max_n = max(self.max_n, int(n.max()))
        return self

    def __len__(self):
        if self.items is not None:
            return len(self.items)
        return len(self._items) + sum(len(c) for c in getattr(self, "_item_chunks", []))

    def aligned(self, elems: int) -> bool:
        """All A/B/C offsets are multiples of ``elems`` elements."""
        return self._align % elems == 0

    def finalize(self):
        if self.items is None:
            chunks_i = getattr(self, "_item_chunks", [])
            chunks_k = getattr(self, "_kp_chunks", [])
            if chunks_i:
                if self._items:
                    raise RuntimeError("GemmBatch: mixing add() after add_arrays() is not supported")
                self.items = np.concatenate(chunks_i)
                self.kpairs = np.concatenate(chunks_k) if sum(len(c) for c in chunks_k) else np.zeros(1, dtype=KPAIR)
                self._item_chunks = self._kp_chunks = []
            else:
                self.items = np.array(self._items, dtype=GEMM_ITEM)
                self.kpairs = np.array(self._kps if self._kps else [(0, 0, 0, 0)], dtype=KPAIR)
            self._items = self._kps = None
        return self

    def device_arrays(self, device):
        self.finalize()
        return _pred(self._upload(self.items, device)), self._upload(self.kpairs, device)


class TileBatch(_Uploadable):
    """List of tiles (a_off, b_off, m, n, global row, global col) for map/trsm/norm launches."""

    def __init__(self):
        super().__init__()
        self._items = []
        self.items = None
        self.max_m = self.max_n = 0

    def add(self, a_off: int, m: int, n: int, gi: int = 0, gj: int = 0, b_off: int = 0):
        self._items.append((a_off, b_off, m, n, gi, gj))
        self.max_m = max(self.max_m, m)
        self.max_n = max(self.max_n, n)
        return self

    def __len__(self):
        return len(self._items) if self.items is None else len(self.items)

    def finalize(self):
        if self.items is None:
            self.items = np.array(self._items if self._items else [], dtype=TILE_ITEM)
            self._items = None
        return self

    def device_array(self, device):
        self.finalize()
        return _pred(self._upload(self.items, device))
