"""Python side of the C ABI (``capi/libdplasma.so``, header ``capi/include/dplasma.h``).

The C library embeds the interpreter and forwards every ``dplasma_<p><op>(ctx, ...)`` call here:
descriptors are handles to :class:`~dplasma_amd.descriptor.TiledMatrix` objects, enums are the
reference's integer values (``src/include/dplasma/constants.h``), scalars arrive as doubles
(complex as re/im pairs).  Host matrices enter and leave descriptors through LAPACK-layout
(column-major, ``lda``) buffers -- the role of ``dplasma_zlacpy`` from/to a 1x1 LAPACK
descriptor in the reference tests (``tests/testing_zgemm.c:200-287``).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import api as _api
from .constants import PREC_DTYPE
from .context import init as _init

_PREC_BY_CODE = {2: "s", 3: "d", 4: "c", 5: "z"}   # dplasmaRealFloat .. dplasmaComplexDouble
_NP = {"s": np.float32, "d": np.float64, "c": np.complex64, "z": np.complex128}


def init(nb_cores: int, gpus: int):
    dev = os.environ.get("DPLASMA_DEVICE")
    if dev is None and gpus == 0:
        dev = "cpu"
    return _init(nb_cores=nb_cores if nb_cores > 0 else None, device=dev, gpus=gpus if gpus >= 0 else None)


def fini(ctx):
    from .context import fini as _fini
    _fini(ctx)


def desc_block_cyclic(ctx, prec_code: int, mb: int, nb: int, m: int, n: int, P: int, Q: int, uplo: int):
    from .descriptor import TiledMatrix
    p = _PREC_BY_CODE[prec_code]
    if P <= 0:
        P = ctx.P
    if Q <= 0:
        Q = ctx.world // P
    return TiledMatrix(PREC_DTYPE[p], mb, nb, m, n, P=P, Q=Q, rank=ctx.rank, device=ctx.device, uplo=uplo)


def desc_int(ctx, mb: int, nb: int, m: int, n: int, P: int, Q: int):
    """Integer descriptor (pivots): same layout rules as the numeric ones."""
    from .descriptor import TiledMatrix
    if P <= 0:
        P = ctx.P
    if Q <= 0:
        Q = ctx.world // P
    return TiledMatrix(torch.int32, mb, nb, m, n, P=P, Q=Q, rank=ctx.rank, device=ctx.device)


def _host_view(desc, addr: int, lda: int):
    np_t = _NP.get(desc.prec, np.int32)
    item = np.dtype(np_t).itemsize
    nbytes = lda * max(desc.n, 1) * item
    buf = (ctypes.c_char * nbytes).from_address(addr)
    a = np.frombuffer(buf, dtype=np_t).reshape(max(desc.n, 1), lda)   # row c = column c
    return a


def desc_set_lapack(desc, addr: int, lda: int) -> int:
    """Scatter a host column-major m x n matrix (leading dimension lda) into the local tiles."""
    a = _host_view(desc, addr, lda)
    dense = torch.from_numpy(np.ascontiguousarray(a[:desc.n, :desc.m].T))
    desc.from_dense(dense)
    return 0


def desc_get_lapack(desc, addr: int, lda: int) -> int:
    """Copy the local tiles into a host column-major buffer (zeros where another rank owns the tile)."""
    a = _host_view(desc, addr, lda)
    dense = desc.to_dense_local().numpy()
    a[:desc.n, :desc.m] = dense.T
    return 0


# ----------------------------------------------------------------------------- taskpools
def new(ctx, name: str, *args):
    """dplasma_<p><op>_New(ctx, args...) -> the taskpool (nothing runs yet)."""
    return getattr(_api, name + "_New")(ctx, *args)


def destruct(tp) -> int:
    d = getattr(tp, "destruct", None)
    if d is not None:
        d()
    return 0


def add_taskpool(ctx, tp) -> int:
    ctx.add_taskpool(tp)
    return 0


def start(ctx) -> int:
    ctx.start()
    return 0


def wait(ctx) -> int:
    ctx.wait()
    return 0


def tp_result(tp) -> int:
    r = getattr(tp, "result", None)
    return int(r) if isinstance(r, (int, float, bool)) else 0


# ----------------------------------------------------------------------------- caller-owned memory
class _DevArray:
    """__cuda_array_interface__ view of a raw device pointer (zero-copy torch.as_tensor)."""

    _TYPESTR = {torch.float32: "<f4", torch.float64: "<f8", torch.complex64: "<c8", torch.complex128: "<c16",
                torch.int32: "<i4"}

    def __init__(self, addr: int, count: int, dtype: torch.dtype):
        self.__cuda_array_interface__ = {"shape": (count,), "typestr": self._TYPESTR[dtype],
                                         "data": (int(addr), False), "version": 2}


class _HipPtrAttr(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int), ("devicePointer", ctypes.c_void_p),
                ("hostPointer", ctypes.c_void_p), ("isManaged", ctypes.c_int), ("allocationFlags", ctypes.c_uint)]


_HIP = None


def ptr_is_device(addr: int) -> bool:
    """hipPointerGetAttributes: device / managed memory of a GPU (plain host memory -> False)."""
    global _HIP
    if not addr or not torch.cuda.is_available():
        return False
    if _HIP is None:
        _HIP = ctypes.CDLL("libamdhip64.so")
    a = _HipPtrAttr()
    rc = _HIP.hipPointerGetAttributes(ctypes.byref(a), ctypes.c_void_p(addr))
    if rc != 0:
        _HIP.hipGetLastError()
        return False
    return a.type in (2, 3)


def wrap_memory(ctx, addr: int, count: int, dtype: torch.dtype, on_device=None):
    """(tensor, writeback) over `count` elements at `addr`: device memory of the context's GPU is
    used in place; host memory is used in place on a CPU context and staged through the GPU
    (writeback copies the result home) on a GPU context."""
    if on_device is None:
        on_device = ptr_is_device(addr)
    if on_device:
        return torch.as_tensor(_DevArray(addr, count, dtype), device=ctx.device), (lambda: None)
    np_t = {torch.float32: np.float32, torch.float64: np.float64, torch.complex64: np.complex64,
            torch.complex128: np.complex128, torch.int32: np.int32}[dtype]
    nbytes = count * np.dtype(np_t).itemsize
    host = torch.from_numpy(np.frombuffer((ctypes.c_char * nbytes).from_address(addr), dtype=np_t))
    if not ctx.is_gpu:
        return host, (lambda: None)
    dev = host.to(ctx.device)
    return dev, (lambda: host.copy_(dev.cpu()))


def desc_lapack(ctx, prec_code: int, mb: int, nb: int, m: int, n: int, P: int, Q: int, ip: int, jq: int,
                addr: int, lld: int, on_device: int):
    """Descriptor over caller-owned ScaLAPACK-layout local memory (zero copy on the device)."""
    from .constants import STORAGE_LAPACK
    from .descriptor import TiledMatrix
    from .scalapack import numroc
    p = _PREC_BY_CODE[prec_code]
    P = P if P > 0 else ctx.P
    Q = Q if Q > 0 else ctx.world // P
    myrow, mycol = ctx.rank // Q, ctx.rank % Q
    nloc = numroc(n, nb, mycol, jq, Q)
    if bool(on_device) != ctx.is_gpu:
        raise ValueError("desc_lapack: the memory must live where the context computes (device memory on a "
                         "GPU context, host memory on a CPU one); use dplasma_desc_set_lapack to copy")
    data, _ = wrap_memory(ctx, addr, max(1, lld * max(nloc, 1)), PREC_DTYPE[p], on_device=bool(on_device))
    return TiledMatrix(PREC_DTYPE[p], mb, nb, m, n, P=P, Q=Q, ip=ip, jq=jq, rank=ctx.rank, device=data.device,
                       storage=STORAGE_LAPACK, lld=lld, data=data, name="user")


# ----------------------------------------------------------------------------- ScaLAPACK F77 layer
_F77_CTX = None


def _f77_ctx():
    global _F77_CTX
    if _F77_CTX is None:
        from . import context
        _F77_CTX = context._DEFAULT or _init(device=os.environ.get("DPLASMA_DEVICE"))
    return _F77_CTX


def blacs_pinfo():
    c = _f77_ctx()
    return c.rank, c.world


def gridinit_ctx(ctx) -> int:
    from .scalapack import blacs_gridinit
    return blacs_gridinit(ctx)


def blacs_gridinfo(ictxt: int):
    from .scalapack import blacs_gridinfo as _gi
    try:
        return _gi(ictxt)
    except KeyError:
        return (-1, -1, -1, -1)


def _local_count(ctx, desc):
    from .scalapack import numroc
    Q = ctx.Q
    nloc = numroc(desc[3], desc[5], ctx.rank % Q, desc[7], Q)
    return max(1, desc[8] * max(nloc, 1))


def _local_rows(ctx, desc):
    from .scalapack import numroc
    return numroc(desc[2], desc[4], ctx.rank // ctx.Q, desc[6], ctx.P)


def f77_tuple(args) -> int:
    return f77(*args)


def f77(name: str, *args) -> int:
    """One ScaLAPACK-style call from capi/dplasma_f77.cpp (arrays arrive as addresses)."""
    from . import scalapack as sl
    global _F77_CTX
    if name == "init":
        _f77_ctx()
        return 0
    if name == "fini":
        if _F77_CTX is not None:
            from .context import fini as _fini
            _fini(_F77_CTX)
            _F77_CTX = None
        return 0
    if name == "gridinit":
        ctx = _f77_ctx()
        nprow, npcol = args
        if nprow * npcol != ctx.world or nprow != ctx.P:
            from .context import Context
            ctx = Context(device=ctx.device, P=nprow, Q=npcol)
        return sl.blacs_gridinit(ctx)
    prec, op = name[1], name[2:]
    dt = PREC_DTYPE[prec]
    fn = getattr(sl, name)

    def arr(addr, desc):
        ctx = sl._CTXTS[desc[1]]
        return wrap_memory(ctx, addr, _local_count(ctx, desc), dt)

    if op == "gemm_":
        ta, tb, m, n, k, alpha, a, ia, ja, da, b, ib, jb, db, beta, c, ic, jc, dc = args
        A, _ = arr(a, da)
        B, _ = arr(b, db)
        C, wb = arr(c, dc)
        fn(ta, tb, m, n, k, alpha, A, ia, ja, da, B, ib, jb, db, beta, C, ic, jc, dc)
        wb()
        return 0
    if op == "potrf_":
        uplo, n, a, ia, ja, da = args
        A, wb = arr(a, da)
        info = fn(uplo, n, A, ia, ja, da)
        wb()
        return int(info or 0)
    if op == "getrf_":
        m, n, a, ia, ja, da, ipiv = args
        A, wb = arr(a, da)
        ctx = sl._CTXTS[da[1]]
        npiv = _local_rows(ctx, da) + da[4]
        piv = np.frombuffer((ctypes.c_int32 * npiv).from_address(ipiv), dtype=np.int32) if ipiv else None
        info = fn(m, n, A, ia, ja, da, piv)
        wb()
        return int(info or 0)
    if op in ("trsm_", "trmm_"):
        side, uplo, ta, diag, m, n, alpha, a, ia, ja, da, b, ib, jb, db = args
        A, _ = arr(a, da)
        B, wb = arr(b, db)
        fn(side, uplo, ta, diag, m, n, alpha, A, ia, ja, da, B, ib, jb, db)
        wb()
        return 0
    if op == "latsqr_":
        m, n, a, ia, ja, da, tau = args
        A, wb = arr(a, da)
        tv = None
        if tau:
            tv, twb = wrap_memory(sl._CTXTS[da[1]], tau, max(1, min(m, n)), dt)
        info = fn(m, n, A, ia, ja, da, tau=tv)[0]
        wb()
        if tau:
            twb()
        return int(info or 0)
    raise ValueError(f"unknown ScaLAPACK entry point {name}")


def call(ctx, name: str, *args):
    """Forward one C call: dplasma_<prec><op>(ctx, args...) -> dplasma_amd.<prec><op>(ctx, *args)."""
    fn = getattr(_api, name)
    r = fn(ctx, *args)
    if isinstance(r, bool):
        return int(r)
    if r is None:
        return 0
    if isinstance(r, (int, float)):
        return r
    if isinstance(r, torch.Tensor):
        return float(r.item())
    return 0
