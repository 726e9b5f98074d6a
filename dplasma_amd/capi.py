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
    if name.startswith("x:"):
        return _ext(name[2:], True)(ctx, *args)
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


# ----------------------------------------------------------------------------- extended entry points
# (tools/gen_capi.py EXT: QR-tree handles, caller int arrays, butterfly handles, taskpool setters)
class _CInts:
    """A caller's int array (int *) as a mutable sequence: reads and writes go to the C memory."""

    def __init__(self, addr: int, n: int):
        self._a = (ctypes.c_int * max(1, n)).from_address(addr)
        self._n = n

    def __len__(self):
        return self._n

    def __getitem__(self, i):
        if not -self._n <= i < self._n:
            raise IndexError(i)
        return self._a[i % self._n]

    def __setitem__(self, i, v):
        if not -self._n <= i < self._n:
            raise IndexError(i)
        self._a[i % self._n] = int(v)

    def __iter__(self):
        return (self._a[i] for i in range(self._n))


def _ints(addr: int, n: int):
    return _CInts(addr, n) if addr else None


def _minmnt(A):
    return min(A.mt, A.nt)


def _x_getrf_qrf(new, p):
    def f(ctx, tree, A, IPIV, TS, TT, criteria, alpha, lu_tab, INFO):
        fn = getattr(_api, f"{p}getrf_qrf" + ("_New" if new else ""))
        r = fn(ctx, tree, A, IPIV, TS, TT, criteria, alpha, _ints(lu_tab, _minmnt(A)), _ints(INFO, 1))
        return r
    return f


def _x_trsmpl_qrf(new, p):
    def f(ctx, tree, A, IPIV, B, TS, TT, lu_tab):
        fn = getattr(_api, f"{p}trsmpl_qrf" + ("_New" if new else ""))
        return fn(ctx, tree, A, IPIV, B, TS, TT, _ints(lu_tab, _minmnt(A)))
    return f


# butterfly vectors cross the C ABI as the reference's raw host arrays: level x n values of the precision
# (complex: (re, im) pairs, im = 0), malloc'd by the C side; the framework's own form is a (level, n) real tensor
_BUT_CT = {"s": (ctypes.c_float, 1), "d": (ctypes.c_double, 1), "c": (ctypes.c_float, 2), "z": (ctypes.c_double, 2)}


def _but_in(p, addr, level, n):
    """The (level, n) float64 tensor of a caller's butterfly vector at address addr (None: no butterfly)."""
    if not addr or level <= 0:
        return None
    ct, comp = _BUT_CT[p]
    raw = np.ctypeslib.as_array((ct * (level * n * comp)).from_address(int(addr)))
    return torch.from_numpy(raw[::comp].astype(np.float64).reshape(level, n).copy())


def _but_out(p, U):
    ct, comp = _BUT_CT[p]
    v = U.detach().cpu().to(torch.float64).numpy().reshape(-1)
    out = np.zeros(v.size * comp, dtype=np.float32 if ct is ctypes.c_float else np.float64)
    out[::comp] = v
    return out.tobytes()


def _x_hebut(new, p):
    def f(ctx, A, level):
        return _but_out(p, getattr(_api, f"{p}hebut")(ctx, A, levels=int(level)))
    return f


def _x_hetrs(new, p):
    def f(ctx, uplo, A, B, U_but, level):
        return getattr(_api, f"{p}hetrs")(ctx, A, B, U_but=_but_in(p, U_but, int(level), B.m))
    return f


def _x_gebut(new, p):
    def f(ctx, A, U_but, level):
        return getattr(_api, f"{p}gebut")(ctx, A, _but_in(p, U_but, int(level), A.n))
    return f


def _x_gebmm(new, p):
    def f(ctx, A, U_but, level, trans):
        return getattr(_api, f"{p}gebmm")(ctx, A, _but_in(p, U_but, int(level), A.m), trans)
    return f


def _x_gebrd_ge2gbx(new, p):
    # the reference's R-bidiag pre-QR (qrtre0, TS0 / TT0) is not performed here: TS0 / TT0 hold the QR
    # block factors and TS / TT the LQ ones (models/eigen.py gebrd_ge2gbx_New)
    def f(ctx, ib, qrtre0, qrtree, lqtree, A, TS0, TT0, TS, TT, Band):
        fn = getattr(_api, f"{p}gebrd_ge2gbx" + ("_New" if new else ""))
        r = fn(ctx, ib, qrtree if qrtree is not None else qrtre0, lqtree, A, TS0, TT0, TS, TT, Band)
        return r if new else 0
    return f


def _x_lanm2(new, p):
    def f(ctx, A, info):   # *info: the power iterations run (negative: not converged)
        lst = []
        v = float(getattr(_api, f"{p}lanm2")(ctx, A, info=lst))
        iv = _ints(info, 1)
        if iv is not None and lst:
            iv[0] = lst[0]
        return v
    return f


def _x_print(new, p):
    def f(ctx, uplo, A):
        return getattr(_api, f"{p}print")(ctx, uplo, A)
    return f


_EXT_ADAPT = {"getrf_qrf": _x_getrf_qrf, "trsmpl_qrf": _x_trsmpl_qrf, "hebut": _x_hebut, "hetrs": _x_hetrs,
              "gebut": _x_gebut, "gebmm": _x_gebmm, "gebrd_ge2gbx": _x_gebrd_ge2gbx, "lanm2": _x_lanm2,
              "print": _x_print}


def _ext(pname: str, new: bool):
    p, op = pname[0], pname[1:]
    ad = _EXT_ADAPT.get(op)
    if ad is not None:
        return ad(new, p)
    return getattr(_api, pname + ("_New" if new else ""))


def call_obj(ctx, name: str, *args):
    """An extended entry point returning a framework object to C (an opaque handle)."""
    return _ext(name[2:] if name.startswith("x:") else name, False)(ctx, *args)


def tp_setter(tp, name: str, v: int) -> int:
    """dplasma_<p>potrf_setrecursive / geqrf_setrecursive on a framework taskpool."""
    op = name[2:] if name.startswith("x:") else name
    getattr(_api, op)(tp, int(v))
    return 0


def qrtree_init(kind: str, trans: int, A, ints):
    """dplasma_hqr_init / systolic_init / svd_init (qr_param.h:120-148) -> the tree object."""
    from .models import qrtree as qt
    ints = [int(x) for x in ints]
    if kind == "hqr":
        llvl, hlvl, a, p, domino, tsrr = ints
        return qt.hqr_init(trans, A, llvl=llvl, hlvl=hlvl, a=a, p=p if p > 0 else None, domino=bool(domino),
                           tsrr=bool(tsrr))
    if kind == "systolic":
        return qt.systolic_init(trans, A, p=ints[0], q=ints[1])
    if kind == "svd":
        return qt.svd_init(trans, A, hlvl=ints[0], p=ints[1], nbcores_per_node=ints[2], ratio=ints[3])
    raise ValueError(kind)


def qrtree_check(tree) -> int:
    try:
        return int(tree.check())
    except AssertionError as e:
        print(f"dplasma_qrtree_check: {e}", flush=True)
        return 1


def qrtree_print(tree, what: str, k: int, perm_addr: int, filename: str) -> int:
    """dplasma_qrtree_print_* (qr_param.h debugging functions): text on stdout, DOT to a file."""
    kk = range(min(tree.mt, tree.nt))
    if what == "dag":
        with open(filename or "qrtree.dot", "w") as f:
            f.write(tree.dot())
        return 0
    if what == "type":
        out = tree.print_type()
    elif what == "pivot":
        out = tree.print_pivot()
    elif what == "nbgeqrt":
        out = tree.print_nbgeqrt()
    elif what == "perm":
        # the order in which rows are killed at each step (perm[k * mt + i])
        arr = (ctypes.c_int * (tree.mt * max(1, len(kk)))).from_address(perm_addr) if perm_addr else None
        lines = []
        for k_ in kk:
            order = [k_] + [m for (_, m, _) in reversed(tree.kills(k_))]
            if arr is not None:
                for i, m in enumerate(order):
                    arr[k_ * tree.mt + i] = m
            lines.append(" ".join(str(m) for m in order))
        out = "\n".join(lines)
    elif what in ("next_k", "prev_k"):
        lines = []
        for p_ in range(k, tree.mt):
            f = tree.nextpiv if what == "next_k" else tree.prevpiv
            lines.append(" ".join("%3d" % f(k, p_, m) for m in range(k, tree.mt + 1)))
        out = "\n".join(lines)
    elif what == "geqrt_k":
        out = " ".join(str(m) for m in tree.heads(k))
    else:
        raise ValueError(what)
    print(out, flush=True)
    return 0


def call(ctx, name: str, *args):
    """Forward one C call: dplasma_<prec><op>(ctx, args...) -> dplasma_amd.<prec><op>(ctx, *args)."""
    fn = _ext(name[2:], False) if name.startswith("x:") else getattr(_api, name)
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
