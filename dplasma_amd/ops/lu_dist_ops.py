"""Distributed partial-pivoting panel of the P x Q LU (reference: ``src/zgetrf_ptgpanel.jdf``).

The reference factors a panel spread over the P process rows of its process column with one round of
tasks per column: GETRF_MAX finds each process's |max| (``:206``), GETRF_RDC / GETRF_SVM reduce the P
candidates (``:379-520``) and GETRF_SND exchanges the winner in a log2(P) Bruck pattern (``:522-590``).

Here every rank of the process column holds one column-major panel buffer

    rows [0, tr)   T -- a replica of the diagonal tile rows (every pivot destination is one of them)
    rows [tr, m)   its own panel rows, at panel-relative positions ``lrel``

and factors it with the same recursion as the one-process :class:`~dplasma_amd.ops.tile_ops.PanelLU`
(halves down to 64-column blocks, TRSM + MFMA GEMM joins), except that

* a block picks each column's pivot over the whole process column, and
* an interchange moves FULL panel rows at once (the winner's row arrives with its candidate; the
  displaced row j is a T row, so the rank that takes it already holds it), which makes the recursion's
  laswp steps unnecessary.

Two transports, the same semantics (ties resolved by the smallest position, LAPACK i?amax):

* GPU (``csrc/kernels/lu_dist.hip``): one persistent launch per block; per column one local grid barrier
  and one cross-process hand-off through IPC-mapped exchange buffers (system-scope stores + epoch
  flags over xGMI) -- no host involvement inside a panel.
* host (CPU, or a GPU group whose buffers cannot be IPC-mapped): one all-gather of
  ``(|v|, position, row)`` per column over the process-column group.
"""
from __future__ import annotations

import atexit
import ctypes
import os

import torch
import torch.distributed as dist

from ..constants import dplasmaLeft, dplasmaLower, dplasmaNoTrans, dplasmaUnit
from . import _lib
from .batch import GemmBatch, TileBatch
from .tile_ops import LU_BW, gemm, trsm


def _is_gpu(t: torch.Tensor) -> bool:
    return t.device.type == "cuda"


class PanelXchg:
    """The exchange buffers of one process column: on every rank ``2 x P`` slots (column parity x
    sender) of ``{epoch flag, position, |v|, row[kbw]}``, IPC-mapped by every peer.  ``epoch`` counts
    the panel columns factored so far; it advances identically on every rank of the column."""

    def __init__(self, group, me: int, P: int, kbw: int, dtype: torch.dtype, device, max_rows: int = 0):
        self.group, self.me, self.P, self.kbw = group, me, P, kbw
        self.dtype, self.device = dtype, torch.device(device)
        self.epoch = 1
        self.ok = False
        self._local = None
        self._opened = []
        if self.device.type != "cuda" or not kernel_ok(dtype) or os.environ.get("DPLASMA_LU_XCHG", "ipc") == "host":
            return
        lib = _lib.load()
        self.slot_bytes = int(lib.dpl_lu_dist_slot_bytes(_lib.prec_code(dtype), kbw))
        nbytes = 2 * P * self.slot_bytes
        hb = int(lib.dpl_ipc_handle_bytes())
        handle = (ctypes.c_char * hb)()
        ptr = ctypes.c_void_p()
        torch.cuda.synchronize(self.device)
        # the persistent kernel holds one row per thread on at most one workgroup per CU: a rank whose
        # panel rows exceed that sends the whole column to the host transport (the choice must agree)
        ncu = min(256, torch.cuda.get_device_properties(self.device).multi_processor_count)
        fits = max_rows <= 256 * ncu
        rc = lib.dpl_xchg_alloc(nbytes, ctypes.byref(ptr), handle) if fits else -4
        mine = bytes(handle) if rc == 0 else b""
        allh = [None] * P
        dist.all_gather_object(allh, (rc, mine), group=group)
        if any(r != 0 for r, _ in allh):
            if rc == 0:
                lib.dpl_xchg_free(ptr)
            return                                   # some rank cannot export: host transport everywhere
        self._local = ptr.value
        bases, ok = [], 1
        for q, (_, h) in enumerate(allh):
            if q == me:
                bases.append(self._local)
                continue
            p = ctypes.c_void_p()
            r = lib.dpl_xchg_open(ctypes.create_string_buffer(h, len(h)), ctypes.byref(p))
            if r != 0:
                ok = 0
                bases.append(0)
                continue
            self._opened.append(p.value)
            bases.append(p.value)
        flags = [None] * P
        dist.all_gather_object(flags, ok, group=group)
        if not all(flags):
            self.close()
            return
        self.peers = torch.tensor(bases, dtype=torch.int64).to(self.device)
        self.ok = True

    def close(self):
        """Unmap the peers' buffers and free mine (every rank of the column calls it after the last
        panel has completed on every rank: no peer writes into my buffer any more)."""
        if self._local is None:
            return
        lib = _lib.load()
        torch.cuda.synchronize(self.device)
        dist.barrier(group=self.group)
        for p in self._opened:
            lib.dpl_xchg_close(ctypes.c_void_p(p))
        self._opened = []
        dist.barrier(group=self.group)
        lib.dpl_xchg_free(ctypes.c_void_p(self._local))
        self._local = None
        self.ok = False


_XCHG = {}


def panel_xchg(group, me: int, P: int, kbw: int, dtype: torch.dtype, device, max_rows: int = 0) -> PanelXchg:
    """The exchange buffers of a process column, created once per (group, width, dtype) and re-used by
    every later factorisation (their epochs continue), so repeated LU runs neither re-export IPC
    handles nor leak mappings.  ``release_all()`` frees them (collective over each column group)."""
    dev = torch.device(device)
    ncu = min(256, torch.cuda.get_device_properties(dev).multi_processor_count) if dev.type == "cuda" else 256
    # max_rows is the largest panel of ANY rank (identical everywhere), so every rank picks the same key
    key = (id(group), me, P, kbw, dtype, str(dev), max_rows <= 256 * ncu)
    xc = _XCHG.get(key)
    if xc is None:
        xc = _XCHG[key] = PanelXchg(group, me, P, kbw, dtype, device, max_rows)
    return xc


def release_all():
    """Unmap and free every cached exchange buffer (call on every rank, e.g. before fini)."""
    for key in list(_XCHG):
        _XCHG.pop(key).close()


def _at_exit():
    """Interpreter exit with exchange buffers still cached (a script that never called release_all):
    the peers' IPC mappings must be closed before the HIP runtime's own static teardown runs, or that
    teardown can fault in __cxa_finalize -- what ended a 2-rank rehearsal under rocprofv3 with SIGSEGV
    after its SUCCESS line (round 3, gpurun_out/b2_lud_r0.log).  Collective release while the process
    group lives; otherwise only the local unmapping (my exported buffer goes with the process)."""
    if not _XCHG:
        return
    try:
        if dist.is_available() and dist.is_initialized():
            release_all()
            return
    except Exception:   # a peer already gone: fall through to the local cleanup
        pass
    lib = _lib.load()
    for xc in list(_XCHG.values()):
        for p in xc._opened:
            lib.dpl_xchg_close(ctypes.c_void_p(p))
        xc._opened = []
    _XCHG.clear()


atexit.register(_at_exit)


def _block_host(P, ld, m, c0, cend, kbw, tr, diag, pos, ipiv, info, info_base, xc: PanelXchg):
    """One block of the distributed panel through per-column all-gathers (same arithmetic as the
    one-process CPU lu_block restricted to the block columns, plus whole-row interchanges)."""
    A = torch.as_strided(P, (m, kbw), (1, ld), 0)
    cplx = A.dtype.is_complex
    rdt = A.real.dtype if cplx else A.dtype
    W = 2 + kbw
    xb = torch.zeros(xc.P, W, dtype=A.dtype, device=A.device)
    for j in range(c0, cend):
        lo = j if diag else max(j, tr)
        mine = xb[xc.me]
        mine.zero_()
        mine[0] = -1.0
        loc = -1
        if m > lo:
            col = A[lo:, j]
            c = (col.real.abs() + col.imag.abs()) if cplx else col.abs()
            i = int(torch.argmax(c))
            loc = lo + i
            mine[0] = c[i]
            mine[1] = float(pos[loc])
            mine[2:] = A[loc, :]
        if xc.P > 1:
            from ..parallel import comm
            comm.allgather_inplace(xb, xc.me, xc.group)
        hv = xb[:, :2].real.to(rdt).cpu().tolist() if cplx else xb[:, :2].cpu().tolist()
        qw = max(range(xc.P), key=lambda q: (hv[q][0], -hv[q][1]))
        pw = int(hv[qw][1])
        dest = pw if pw < tr else (loc if qw == xc.me else -1)
        if dest != j:
            old = A[j, :].clone()
            A[j, :] = xb[qw, 2:]
            if dest >= 0:
                A[dest, :] = old
        ipiv[j] = pw
        d = A[j, j]
        if d == 0:
            if int(info[0]) == 0:
                info[0] = info_base + j + 1
        else:
            A[j + 1:, j] /= d
        if j + 1 < cend:
            A[j + 1:, j + 1:cend] -= torch.outer(A[j + 1:, j], A[j, j + 1:cend])
        xc.epoch += 1


class DistPanelLU:
    """Recursive LU with partial pivoting of one panel distributed over a process column (see the
    module docstring).  ``buf`` is this rank's (T + own rows) buffer, ``ld`` >= m rows, ``kb`` columns;
    ``lrel`` the panel-relative positions of the own rows (increasing, all >= tr)."""

    def __init__(self, buf: torch.Tensor, ld: int, m: int, kb: int, tr: int, diag: bool, lrel):
        self.buf, self.ld, self.m, self.kb, self.tr, self.diag = buf, ld, m, kb, tr, bool(diag)
        lrel = [int(x) for x in lrel]
        self.pos = list(range(tr)) + lrel
        self.lrel = torch.tensor(lrel + [0], dtype=torch.int32, device=buf.device)
        self.kf = min(tr, kb)
        self.plan = []
        self._rec(0, self.kf)
        if kb > self.kf:   # wide panel: the columns past the last pivot only get U = L^-1 A
            self.plan.append(("trsm", TileBatch().add(0, self.kf, kb - self.kf, b_off=self.kf * ld).finalize()))
        if _is_gpu(buf):   # device item arrays now (the _New phase), not inside the first run
            from .tile_ops import _trsm_groups
            for op in self.plan:
                if op[0] == "trsm":
                    _trsm_groups(op[1], dplasmaLeft, buf)
                elif op[0] == "gemm":
                    op[1].device_arrays(buf.device)

    def _rec(self, c0: int, n: int):
        ld, m = self.ld, self.m
        if n <= LU_BW:
            self.plan.append(("block", c0, c0 + n))
            return
        n1 = (n // 2 + 15) // 16 * 16
        self._rec(c0, n1)
        c1 = c0 + n1
        self.plan.append(("trsm", TileBatch().add(c0 + c0 * ld, n1, n - n1, b_off=c0 + c1 * ld).finalize()))
        if m > c1:
            gb = GemmBatch().add(c1 + c1 * ld, m - c1, n - n1, [(c1 + c0 * ld, c0 + c1 * ld, n1)]).finalize()
            self.plan.append(("gemm", gb))
        self._rec(c1, n - n1)

    def run(self, ipiv: torch.Tensor, ws: torch.Tensor, cnt: torch.Tensor, info: torch.Tensor, info_base: int,
            xc: PanelXchg):
        Pb, ld, m = self.buf, self.ld, self.m
        gpu = _is_gpu(Pb) and xc.ok
        for op in self.plan:
            if op[0] == "block":
                c0, cend = op[1], op[2]
                if gpu:
                    lib = _lib.load()
                    rc = lib.dpl_lu_block_dist(_lib.prec_code(Pb.dtype), Pb.data_ptr(), ld, m, c0, cend, self.kb,
                                               self.tr, int(self.diag), self.lrel.data_ptr(), ipiv.data_ptr(),
                                               ws.data_ptr(), cnt.data_ptr(), xc.peers.data_ptr(), xc.P, xc.me,
                                               xc.slot_bytes, xc.epoch, info.data_ptr(), int(info_base),
                                               _lib.stream_ptr())
                    _lib.check(rc, "lu_block_dist")
                    xc.epoch += cend - c0
                    us = getattr(xc, "model_us_per_col", 0.0)
                    if us > 0:   # rank replay (tools/replay_lu.py): the cross-rank hand-offs as modelled latency
                        _lib.check(lib.dpl_delay(float(us * (cend - c0)), 1, _lib.stream_ptr()), "delay")
                else:
                    _block_host(Pb, ld, m, c0, cend, self.kb, self.tr, self.diag, self.pos, ipiv, info, info_base,
                                xc)
            elif op[0] == "trsm":
                trsm(dplasmaLeft, dplasmaLower, dplasmaNoTrans, dplasmaUnit, 1.0, Pb, ld, Pb, ld, op[1])
            else:
                gemm(dplasmaNoTrans, dplasmaNoTrans, -1.0, Pb, ld, Pb, ld, 1.0, Pb, ld, op[1])


def dist_workspace(kb: int, device) -> torch.Tensor:
    dev = torch.device(device)
    if dev.type == "cuda":
        return torch.zeros(int(_lib.load().dpl_lu_dist_ws_bytes(kb)) // 8 + 8, dtype=torch.float64, device=dev)
    return torch.zeros(8, dtype=torch.float64)


def kernel_ok(dtype: torch.dtype) -> bool:
    """The persistent exchange kernel covers the real precisions (complex panels use the host path)."""
    return dtype in (torch.float64, torch.float32)


__all__ = ["PanelXchg", "DistPanelLU", "dist_workspace", "kernel_ok", "panel_xchg", "release_all"]
