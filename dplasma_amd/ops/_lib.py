"""ctypes binding of the in-tree HIP kernel library ``lib/libdplasma_kernels.so``.

The library is built by ``tools/build.py`` (``hipcc --offload-arch=gfx950``).
On a GPU box the native path is mandatory: if a CUDA/HIP tensor reaches a
kernel wrapper and the library cannot be loaded we raise instead of silently
falling back to PyTorch/rocBLAS (no vendor-BLAS fallback, BASELINE.json).
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path

import torch

from ..constants import DTYPE_CODE

_LIBDIR = Path(__file__).resolve().parents[1] / "lib"
_LIB = None
_LOCK = threading.Lock()

c_int, c_ll, c_ull, c_vp = ctypes.c_int, ctypes.c_longlong, ctypes.c_ulonglong, ctypes.c_void_p

_SIGS = {
    # device task runtime (dtr.hip): DtrArgs image in device memory, workgroups, stream
    "dpl_dtr_potrf": [c_vp, c_int, c_vp],
    "dpl_dtr_potrf_q": [c_vp, c_int, c_vp],
    "dpl_dtr_args_size": [],
    "dpl_dtr_field": [ctypes.c_char_p],
    # prec, transA, transB, nitems, items, kpairs, max_m, max_n, alpha*, A, lda, B, ldb, beta*, C, ldc, vec_ok, generic, stream
    "dpl_gemm_batched": [c_int, c_int, c_int, c_int, c_vp, c_vp, c_int, c_int, c_vp, c_vp, c_int, c_vp, c_int, c_vp,
                         c_vp, c_int, c_int, c_int, c_vp],
    # prec, uplo, n, A, a_off, lda, info*, info_base, stream
    "dpl_potrf_tile": [c_int, c_int, c_int, c_vp, c_ll, c_int, c_vp, c_int, c_vp],
    # prec, side, uplo, trans, diag, nitems, items, max_m, max_n, alpha*, A, lda, B, ldb, ntri, tri_off, work, stream
    "dpl_trsm_batched": [c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_int, c_int, c_vp, c_vp, c_int, c_vp, c_int,
                         c_int, c_vp, c_vp, c_vp],
    # prec, kind, nitems, items, mmax, nmax, A, lda, gM, seed, bump*, stream
    "dpl_generate": [c_int, c_int, c_int, c_vp, c_int, c_int, c_vp, c_int, c_ll, c_ull, c_vp, c_vp],
    # prec, part, nitems, items, mmax, nmax, alpha*, beta*, A, lda, stream
    "dpl_laset": [c_int, c_int, c_int, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_vp],
    # prec, part, trans, nitems, items, mmax, nmax, alpha*, A, lda, beta*, B, ldb, copy, stream
    "dpl_qr_panel_multi": [c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp],
    "dpl_qr_panel_multi_ws_bytes": [c_int, c_int, c_int, c_int],
    "dpl_qr_panel_item_bytes": [],
    "dpl_copy_transpose": [c_int, c_int, c_vp, c_int, c_int, c_vp, c_int, c_vp, c_int, c_int, c_int, c_vp],
    "dpl_swap_transpose": [c_int, c_int, c_vp, c_int, c_int, c_vp, c_int, c_int, c_vp],
    "dpl_geadd": [c_int, c_int, c_int, c_int, c_vp, c_int, c_int, c_vp, c_vp, c_int, c_vp, c_vp, c_int, c_int, c_vp],
    # prec, part, nitems, items, mmax, nmax, alpha*, A, lda, stream
    "dpl_lascal": [c_int, c_int, c_int, c_vp, c_int, c_int, c_vp, c_vp, c_int, c_vp],
    # prec, m, n, A, a_off, lda, ipiv*, info*, info_base, pivot, stream
    "dpl_getrf_panel": [c_int, c_int, c_int, c_vp, c_ll, c_int, c_vp, c_vp, c_int, c_int, c_vp],
    # prec, dst, src, rows, nrows, ncols, ld_dst, ld_src, stream
    "dpl_row_gather": [c_int, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp],
    # QR / LQ tile kernels on DAG items (csrc/kernels/qr.hip)
    "dpl_geqrt": [c_int, c_int, c_vp, c_int, c_int, c_int, c_vp],
    "dpl_unmqr": [c_int, c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp],
    "dpl_tsqrt": [c_int, c_int, c_vp, c_int, c_int, c_int, c_int, c_vp],
    "dpl_tsmqr": [c_int, c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_vp],
    # prec, nitems, items, max_n, a_tr, v_tr, ib, conjtrans, mode, stream
    "dpl_qr_apply_mfma": [c_int, c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_vp],
    "dpl_qr_apply_mfma_ok": [c_int, c_int, c_int],
    # prec, nitems, items, a_tr, ib, ts, tri, stream
    "dpl_qr_panel_mfma": [c_int, c_int, c_vp, c_int, c_int, c_int, c_int, c_vp],
    # LU incremental pivoting on DAG items (csrc/kernels/lu_incpiv.hip)
    "dpl_getrf_tile": [c_int, c_int, c_vp, c_vp, c_vp],               # prec, n, items, info*, stream
    "dpl_gessm": [c_int, c_int, c_vp, c_int, c_vp],                   # prec, n, items, max_n, stream
    "dpl_ssssm": [c_int, c_int, c_vp, c_int, c_int, c_int, c_vp],     # + ib, NB
    "dpl_tstrf": [c_int, c_int, c_vp, c_int, c_int, c_int, c_vp, c_vp],  # prec, n, items, ib, NB, max_m, info*, stream
    # prec, part, cols, nitems, items, mmax, nmax, D, ldd, B, ldb, stream
    "dpl_diag_scale": [c_int, c_int, c_int, c_int, c_vp, c_int, c_int, c_vp, c_int, c_vp, c_int, c_vp],
    # prec, kind, part, unit, nitems, items, A, lda, out, ostride, stream
    "dpl_tile_norm": [c_int, c_int, c_int, c_int, c_int, c_vp, c_vp, c_int, c_vp, c_int, c_vp],
    # device-resident pivoting LU (lu_piv.hip)
    # prec, A, ld, m, c0, cend, ipiv, ws, cnt, info, info_base, pivot, stream
    "dpl_lu_block": [c_int, c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_vp],
    # prec, A, ld, ca, cb, ipiv, i0, i1, stream
    # prec, A, ld, m, ca, cb, ipiv, i0, i1, info (an out-of-range pivot: -1001, nothing moved), stream
    "dpl_laswp_panel": [c_int, c_vp, c_int, c_int, c_int, c_int, c_vp, c_int, c_int, c_vp, c_vp],
    "dpl_lu_block_ws_bytes": [c_int],
    "dpl_debug_set_phase_mask": [c_int],
    "dpl_potrf_tile_set_kind": [c_int],
    "dpl_potrf_rb_set_trace": [c_vp],
    # dataflow tile POTRF + panel TRSM (potrf_rb.hip): uplo, n, A, lda, info*, info_base, zbuf, stream
    "dpl_potrf_tile_rbz": [c_int, c_int, c_vp, c_int, c_vp, c_int, c_vp, c_vp],
    # uplo, n, A, lda, info, info_base, zbuf, nrb, items, B, ldb, stream: fused tile POTRF + panel TRSM
    "dpl_potrf_trsm_rb": [c_int, c_int, c_vp, c_int, c_vp, c_int, c_vp, c_int, c_vp, c_vp, c_int, c_vp],
    "dpl_potrf_zbuf_size": [],
    "dpl_trsm_rb_prep": [c_int, c_int, c_vp, c_int, c_vp, c_vp],                    # uplo, n, L, ldl, zbuf, stream
    "dpl_trsm_rb": [c_int, c_int, c_vp, c_int, c_vp, c_int, c_vp, c_vp, c_int, c_vp],  # + nrb, items, B, ldb      # debug: per-workgroup phase timestamps of the dataflow kernel    # 0 = dataflow multi-WG (fp64, n <= 512), 1 = single-WG kernel   # tile POTRF phase ablation (tools/gpu/potrf_tile_phases.py)
    # Householder panel (qr_panel.hip): prec, P, ldp, rbl, rstride, M, nc, kf, V, ldv, Tm, ldt, ws, info, stream
    "dpl_qr_panel": [c_int, c_vp, c_int, c_int, c_ll, c_int, c_int, c_int, c_vp, c_int, c_vp, c_int, c_vp, c_vp,
                     c_vp],
    # prec, src, stride, S, L, dst, stream
    "dpl_sum_partials": [c_int, c_vp, c_ll, c_int, c_ll, c_vp, c_vp],
    "dpl_qr_panel_ws_bytes": [c_int, c_int, c_int],
    "dpl_qr_panel_max_rows": [],
    "dpl_qr_panel_set_prof": [c_vp],
    "dpl_qr_panel_set_pred": [c_vp],
    # ipiv, kb, mrel, dst, src, cnt, info, stream
    "dpl_piv_moves": [c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp],
    # prec, gather, A, ld, mb, r0, rowoff, nrt, coloff, ncols, nct, nb, rows, cnt, maxcnt, buf, ldb, info, stream
    "dpl_rows_move": [c_int, c_int, c_vp, c_int, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_int, c_int, c_vp, c_vp,
                      c_int, c_vp, c_int, c_vp, c_vp],
    "dpl_stream_cumask": [c_vp, c_int, c_vp],
    "dpl_stream_destroy": [c_vp],
    "dpl_delay": [ctypes.c_double, c_int, c_vp],
    "dpl_ipiv_shift": [c_vp, c_vp, c_int, c_int, c_vp],
    # random butterfly level (butterfly.hip): prec, side, trans, m, n, size, r, A, si, sj, mb, nb, ld, stream
    "dpl_butterfly": [c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp, c_ll, c_ll, c_int, c_int, c_int, c_vp],
    "dpl_gemm_set_wg_cap": [c_int],
    "dpl_lu_block_set_kind": [c_int],   # pivoting block kernel: 0 tagged exchange, 1 register rows, 2 flat, 3 xcd counters
    # distributed pivoting panel (lu_dist.hip): prec, A, ld, m, c0, cend, kbw, tr, diag, lrel, ipiv, ws, cnt,
    # peers, P, me, slot_bytes, epoch0, info, info_base, stream
    "dpl_lu_block_dist": [c_int, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp,
                          c_int, c_int, c_int, c_int, c_vp, c_int, c_vp],
    "dpl_lu_dist_ws_bytes": [c_int],
    "dpl_lu_dist_set_maxwg": [c_int],
    "dpl_lu_dist_slot_bytes": [c_int, c_int],
    "dpl_xchg_alloc": [c_ll, c_vp, c_vp],
    "dpl_ipc_alloc": [c_ll, c_int, c_vp, c_vp],
    "dpl_memset_sync": [c_vp, c_int, c_ll],
    "dpl_memcpy_sync": [c_vp, c_vp, c_ll],
    "dpl_xchg_open": [c_vp, c_vp],
    "dpl_xchg_close": [c_vp],
    "dpl_xchg_free": [c_vp],
    "dpl_ipc_handle_bytes": [],
    "dpl_rows_perm_col": [c_int, c_vp, c_int, c_int, c_vp, c_int, c_ll, c_int, c_vp, c_int, c_int, c_vp, c_vp,
                          c_vp],
    "dpl_rows_permute": [c_int, c_vp, c_int, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_int, c_int, c_vp, c_vp, c_vp,
                         c_int, c_vp, c_vp],
    # cross-process-row interchanges: dst, src, cnt, r0, mb, prow, nrt, me, P, ldx, xo, info, stream
    "dpl_rows_xord": [c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp],
    # prec, pack, tmp, ldb, W, xo, cnt, maxcnt, bufs, ldx, stream
    "dpl_rows_xcopy": [c_int, c_int, c_vp, c_int, c_int, c_vp, c_vp, c_int, c_vp, c_int, c_vp],
}
_OPTIONAL = set()
_RESTYPE = {"dpl_dtr_field": c_ll}


def lib_path() -> Path:
    # DPLASMA_KERNELS_LIB: an alternative build of the kernel library (A/B measurements of kernel variants)
    alt = os.environ.get("DPLASMA_KERNELS_LIB")
    return Path(alt) if alt else _LIBDIR / "libdplasma_kernels.so"


def load(build_if_missing: bool = True):
    """Load (building first if needed) the kernel library; returns the CDLL."""
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is not None:
            return _LIB
        p = lib_path()
        if not p.exists() and build_if_missing and os.environ.get("DPLASMA_NO_BUILD") != "1":
            import importlib.util
            spec = importlib.util.spec_from_file_location("dplasma_build", _LIBDIR.parents[1] / "tools" / "build.py")
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            mod.build_kernels()
        lib = ctypes.CDLL(str(p))
        for name, args in _SIGS.items():
            try:
                f = getattr(lib, name)
            except AttributeError:
                if name in _OPTIONAL:
                    continue
                raise
            f.argtypes = args
            f.restype = _RESTYPE.get(name, c_int)
        _LIB = _Declared(lib)
        # pivoting block kernel: LDS tile (default) or register-resident rows (DPLASMA_LU_BLOCK=reg,
        # measured slower: profiles/r3_lu_block_reg.txt)
        _LIB.dpl_lu_block_set_kind({"reg": 1, "flat": 2, "xcd": 3}.get(os.environ.get("DPLASMA_LU_BLOCK", "lds"), 0))
        return _LIB


class _Declared:
    """Exposes only the exports listed in _SIGS: calling an export without a
    declared signature would pass 64-bit pointers as C ints."""

    def __init__(self, lib):
        self._lib = lib

    def __getattr__(self, name):
        if name not in _SIGS:
            raise AttributeError(f"{name}: no ctypes signature declared in dplasma_amd/ops/_lib.py")
        return getattr(self._lib, name)


def available() -> bool:
    try:
        load()
        return True
    except Exception:
        return False


def stream_ptr(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


class Scalar:
    """Host-side scalar of a given dtype, passed by pointer (complex = 2 reals)."""

    __slots__ = ("buf",)

    def __init__(self, value, dtype: torch.dtype):
        if dtype in (torch.complex64, torch.complex128):
            v = complex(value)
            t = ctypes.c_float if dtype == torch.complex64 else ctypes.c_double
            self.buf = (t * 2)(v.real, v.imag)
        elif dtype == torch.float32:
            self.buf = ctypes.c_float(float(value.real if isinstance(value, complex) else value))
        else:
            self.buf = ctypes.c_double(float(value.real if isinstance(value, complex) else value))

    @property
    def ptr(self):
        # NOTE: the Scalar object must stay referenced until the C call returns;
        # callers bind it to a local name first (a temporary may be collected
        # and its buffer reused before the launcher dereferences it).
        return ctypes.c_void_p(ctypes.addressof(self.buf))


def prec_code(dtype: torch.dtype) -> int:
    return DTYPE_CODE[dtype]


def check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"dplasma_amd kernel {what} failed with code {rc}")
