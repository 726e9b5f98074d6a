"""Public API: ``op``, ``op_New``, ``op_Destruct`` and precision-prefixed aliases.

Mirrors ``src/include/dplasma/dplasma_z.h:18-353``: e.g. ``dpotrf(ctx, uplo, A)``
is the blocking call (returns info), ``dpotrf_New`` returns a taskpool that can
be queued with other taskpools before one ``ctx.wait()``, ``dpotrf_Destruct``
releases it.  The precision prefix is checked against the descriptor dtype.
"""
from __future__ import annotations

import functools

from .constants import DTYPE_PREC, dplasmaLeft, dplasmaNoTrans, dplasmaNonUnit, dplasmaUpper
from .models import aux as _aux
from .models import blas3 as _blas3
from .models import cholesky as _chol
from .models import lu as _lu
from .models import generators as _gen
from .models import lu_incpiv as _lui
from .models import qr as _qr
from .models import qrtree as _qrtree
from .models import check as _check
from .models import gemm as _gemm
from .models import potrf as _potrf
from .models import redistribute as _redis

__all__ = []

# generic (precision-agnostic) entry points
_GENERIC = {
    "potrf": _potrf.potrf, "potrf_New": _potrf.potrf_New,
    "gemm": _gemm.gemm, "gemm_New": _gemm.gemm_New,
    "plrnt": _aux.plrnt, "plrnt_New": _aux.plrnt_New,
    "plghe": _aux.plghe, "plghe_New": _aux.plghe_New,
    "plgsy": _aux.plgsy, "plgsy_New": _aux.plgsy_New,
    "laset": _aux.laset, "laset_New": _aux.laset_New,
    "lacpy": _aux.lacpy, "lacpy_New": _aux.lacpy_New,
    "geadd": _aux.geadd, "geadd_New": _aux.geadd_New,
    "tradd": _aux.tradd,
    "lascal": _aux.lascal, "lascal_New": _aux.lascal_New,
    "lange": _aux.lange, "lansy": _aux.lansy, "lanhe": _aux.lanhe, "lantr": _aux.lantr,
    "lanm2": _aux.lanm2, "print": _aux.print_matrix, "apply": _aux.apply, "map2": _aux.map2,
    "pltmg": _gen.pltmg, "latms": _gen.latms,
    "check_potrf": _check.check_potrf, "check_axmb": _check.check_axmb,
    "redistribute": _redis.redistribute,
    "trsm": _blas3.trsm, "trsm_New": _blas3.trsm_New,
    "trmm": _blas3.trmm, "trmm_New": _blas3.trmm_New,
    "symm": _blas3.symm, "symm_New": _blas3.symm_New,
    "hemm": _blas3.hemm, "hemm_New": _blas3.hemm_New,
    "syrk": _blas3.syrk, "syrk_New": _blas3.syrk_New,
    "herk": _blas3.herk, "herk_New": _blas3.herk_New,
    "syr2k": _blas3.syr2k, "syr2k_New": _blas3.syr2k_New,
    "her2k": _blas3.her2k, "her2k_New": _blas3.her2k_New,
    "gerc": _blas3.gerc, "gerc_New": _blas3.gerc_New,
    "geru": _blas3.geru, "geru_New": _blas3.geru_New,
    "potrs": _chol.potrs, "potrs_New": _chol.potrs_New,
    "posv": _chol.posv, "posv_New": _chol.posv_New,
    "trtri": _chol.trtri, "trtri_New": _chol.trtri_New,
    "lauum": _chol.lauum, "lauum_New": _chol.lauum_New,
    "potri": _chol.potri, "potri_New": _chol.potri_New,
    "poinv": _chol.poinv, "poinv_New": _chol.poinv_New,
    "compose": _chol.compose,
    "getrf_nopiv": _lu.getrf_nopiv, "getrf_nopiv_New": _lu.getrf_nopiv_New,
    "getrf_1d": _lu.getrf_1d, "getrf_1d_New": _lu.getrf_1d_New, "getrf": _lu.getrf,
    "laswp": _lu.laswp, "getrs": _lu.getrs, "gesv_1d": _lu.gesv_1d, "gesv": _lu.gesv_1d,
    "getrs_nopiv": _lu.getrs_nopiv, "gesv_nopiv": _lu.gesv_nopiv,
    "ipiv_descriptor": _lu.ipiv_descriptor,
    "getrf_ptgpanel": _lu.getrf_ptgpanel, "getrf_ptgpanel_New": _lu.getrf_ptgpanel_New,
    "trsmpl_ptgpanel": _lu.trsmpl_ptgpanel, "ptgpanel_ipiv_descriptor": _lu.ptgpanel_ipiv_descriptor,
    "gerfs": _lu.gerfs,
    # LU with incremental pivoting
    "getrf_incpiv": _lui.getrf_incpiv, "getrf_incpiv_New": _lui.getrf_incpiv_New,
    "trsmpl_incpiv": _lui.trsmpl_incpiv, "trsmpl_incpiv_New": _lui.trsmpl_incpiv_New,
    "gesv_incpiv": _lui.gesv_incpiv,
    "incpiv_L_descriptor": _lui.L_descriptor, "incpiv_ipiv_descriptor": _lui.ipiv_descriptor,
    # QR / LQ (flat trees)
    "geqrf": _qr.geqrf, "geqrf_New": _qr.geqrf_New, "gelqf": _qr.gelqf, "gelqf_New": _qr.gelqf_New,
    "unmqr": _qr.unmqr, "unmqr_New": _qr.unmqr_New, "unmlq": _qr.unmlq, "unmlq_New": _qr.unmlq_New,
    "ungqr": _qr.ungqr, "ungqr_New": _qr.ungqr_New, "unglq": _qr.unglq, "unglq_New": _qr.unglq_New,
    "geqrs": _qr.geqrs, "gelqs": _qr.gelqs, "gels": _qr.gels,
    # hierarchical QR / LQ (reduction trees)
    "geqrf_param": _qr.geqrf_param, "geqrf_param_New": _qr.geqrf_param_New,
    "gelqf_param": _qr.gelqf_param, "gelqf_param_New": _qr.gelqf_param_New,
    "unmqr_param": _qr.unmqr_param, "unmqr_param_New": _qr.unmqr_param_New,
    "unmlq_param": _qr.unmlq_param, "unmlq_param_New": _qr.unmlq_param_New,
    "ungqr_param": _qr.ungqr_param, "ungqr_param_New": _qr.ungqr_param_New,
    "unglq_param": _qr.unglq_param, "unglq_param_New": _qr.unglq_param_New,
    "geqrs_param": _qr.geqrs_param, "gelqs_param": _qr.gelqs_param,
}


def _destruct(tp):
    if tp is not None:
        tp.destruct()


def _register(name, fn):
    globals()[name] = fn
    __all__.append(name)


def _prec_checked(prec, fn):
    @functools.wraps(fn)
    def wrapper(ctx, *args, **kw):
        for a in args:
            dt = getattr(a, "dtype", None)
            if dt is not None and hasattr(a, "mb"):
                if DTYPE_PREC.get(dt) != prec:
                    raise TypeError(f"{prec}{fn.__name__}: descriptor {a.name} has precision {DTYPE_PREC.get(dt)}")
                break
        return fn(ctx, *args, **kw)
    return wrapper


def register_op(name, fn):
    """Register a generic op and its s/d/c/z aliases (+ _Destruct for _New ops)."""
    _register(name, fn)
    if name.endswith("_New"):
        base = name[:-4]
        _register(base + "_Destruct", _destruct)
    for p in "sdcz":
        alias = p + name
        _register(alias, _prec_checked(p, fn))
        if name.endswith("_New"):
            _register(p + name[:-4] + "_Destruct", _destruct)


for _n, _f in _GENERIC.items():
    register_op(_n, _f)

# precision-independent helpers (QR trees: src/include/dplasma/qr_param.h)
for _n in ("hqr_init", "systolic_init", "svd_init", "qrtree_check", "QRTree", "HQRTree", "SystolicTree", "SVDTree",
           "FlatTree", "FLAT_TREE", "GREEDY_TREE", "FIBONACCI_TREE", "BINARY_TREE", "GREEDY1P_TREE"):
    _register("dplasma_" + _n if _n.endswith("_TREE") else _n, getattr(_qrtree, _n))

# LAWN-263 matrix type codes (src/include/dplasma/constants.h:163-207)
for _n in dir(_gen):
    if _n.startswith("dplasmaMatrix"):
        _register(_n, getattr(_gen, _n))

# DTD insert-task front end (parsec_dtd_* surface) and the DTD Cholesky (src/dtd_wrappers/zpotrf.c)
from .runtime import dtd  # noqa: E402
from .models import dtd_potrf as _dtdp  # noqa: E402
register_op("potrf_dtd", _dtdp.potrf_dtd)
register_op("potrf_dtd_New", _dtdp.potrf_dtd_New)
register_op("potrf_dtd_untied", _dtdp.potrf_dtd_untied)
register_op("gemm_dtd", _dtdp.gemm_dtd)
register_op("gemm_dtd_New", _dtdp.gemm_dtd_New)
register_op("potrf_dtd_untied_New", _dtdp.potrf_dtd_untied_New)
# DTD tile QR and incremental-pivoting LU (tests/testing_zgeqrf_dtd[_untied].c, testing_zgetrf_incpiv_dtd.c)
from .models import dtd_factor as _dtdf  # noqa: E402
for _n in ("geqrf_dtd", "geqrf_dtd_New", "geqrf_dtd_untied", "geqrf_dtd_untied_New", "getrf_incpiv_dtd",
           "getrf_incpiv_dtd_New"):
    register_op(_n, getattr(_dtdf, _n))
for _n in ("taskpool_new", "tile_of", "INPUT", "OUTPUT", "INOUT", "AFFINITY", "VALUE", "SCRATCH", "PUSHOUT"):
    _register("dtd_" + _n, getattr(dtd, _n))
_register("dtd", dtd)

# ScaLAPACK-compatible shims (src/scalapack_wrappers): dp.scalapack.pdgemm_ ...
from . import scalapack  # noqa: E402
_register("scalapack", scalapack)

# LDL^H without pivoting + random butterfly transformation (src/zhetrf.jdf, zhebut/zgebut/zgebmm, ztrdsm, ztrmdm)
from .models import ldl as _ldl  # noqa: E402
for _n, _f in (("hetrf", _ldl.hetrf), ("hetrf_New", _ldl.hetrf_New), ("trdsm", _ldl.trdsm),
               ("trdsm_New", _ldl.trdsm_New), ("trmdm", _ldl.trmdm), ("trmdm_New", _ldl.trmdm_New),
               ("hetrs", _ldl.hetrs), ("hebut", _ldl.hebut), ("gebut", _ldl.gebut), ("gebmm", _ldl.gebmm)):
    register_op(_n, _f)
_register("butterfly_vectors", _ldl.butterfly_vectors)

# Eigenvalues / singular values: two-sided band reductions (src/zherbt_*.jdf, zgebrd_ge2gb.jdf), band ->
# tridiagonal bulge chase (src/zhbrdt.jdf, native C++), heev NoVec driver (src/zheev_wrapper.c)
from .models import eigen as _eig  # noqa: E402
for _n, _f in (("herbt", _eig.herbt), ("herbt_New", _eig.herbt_New), ("heev", _eig.heev), ("heev_New", _eig.heev_New),
               ("gebrd_ge2gb", _eig.gebrd_ge2gb), ("gebrd_ge2gb_New", _eig.gebrd_ge2gb_New),
               ("gebrd_ge2gbx", _eig.gebrd_ge2gbx), ("gebrd_ge2gbx_New", _eig.gebrd_ge2gbx_New)):
    register_op(_n, _f)
for _n in ("hbrdt", "diag_band_to_rect", "sterf", "band_singular_values", "eigvalsh", "gesvd_values"):
    _register(_n, getattr(_eig, _n))
_register("eigen_T", _eig.T_descriptor)

# Tracing / profiling (PaRSEC profiling + --dot + DPLASMA_TRACE_KERNELS analogues) and dplasma_info_t options
from .utils import trace as _trace  # noqa: E402
from .utils import info as _info  # noqa: E402
for _n in ("profiling_start", "profiling_stop", "Tracer"):
    _register(_n, getattr(_trace, _n))


def dot_start(ctx, path):
    """Append the DOT graph of every tile DAG compiled from now on to ``path`` (``--dot``)."""
    open(path, "w").close()
    ctx.dot_file = path


def dot_stop(ctx):
    ctx.dot_file = None


_register("dot_start", dot_start)
_register("dot_stop", dot_stop)
_register("Info", _info.Info)
_register("info_create", _info.info_create)
for _n in ("set", "get", "get_nkeys", "get_nthkey", "delete", "free"):
    _register("info_" + _n, (lambda m: (lambda inf, *a: getattr(inf, m)(*a)))(_n))

# Hybrid LU-QR (src/zgetrf_qrf.jdf, ztrsmpl_qrf.jdf, include/dplasma/lu_qr.h criteria)
from .models import lu_qr as _luqr  # noqa: E402
for _n, _f in (("getrf_qrf", _luqr.getrf_qrf), ("getrf_qrf_New", _luqr.getrf_qrf_New),
               ("trsmpl_qrf", _luqr.trsmpl_qrf), ("trsmpl_qrf_New", _luqr.trsmpl_qrf_New),
               ("gesv_qrf", _luqr.gesv_qrf)):
    register_op(_n, _f)
_register("qrf_ipiv_descriptor", _luqr.qrf_ipiv_descriptor)
for _n in ("DEFAULT_CRITERIUM", "HIGHAM_CRITERIUM", "MUMPS_CRITERIUM", "LU_ONLY_CRITERIUM", "QR_ONLY_CRITERIUM",
           "RANDOM_CRITERIUM", "HIGHAM_SUM_CRITERIUM", "HIGHAM_MAX_CRITERIUM", "HIGHAM_MOY_CRITERIUM"):
    _register(_n, getattr(_luqr, _n))

# Memory-bounded GEMM with host-resident operands (src/zgemm_NN_gpu.jdf)
from .models import gemm_ooc as _gooc  # noqa: E402
register_op("gemm_gpu", _gooc.gemm_gpu)
register_op("gemm_gpu_New", _gooc.gemm_gpu_New)

# GER (src/zger.jdf), HETRD = h2b + b2s (src/zhetrd_wrapper.c), setrecursive hints
from .models import blas3 as _b3  # noqa: E402
for _n in ("gerc", "gerc_New", "geru", "geru_New"):
    register_op(_n, getattr(_b3, _n))
register_op("ger", _b3.geru)
register_op("ger_New", _b3.geru_New)
for _n in ("hetrd", "hetrd_h2b_New", "hetrd_b2s"):
    register_op(_n, getattr(_eig, _n))


def _setrecursive(tp, hnb):
    """dplasma_z{potrf,geqrf}_setrecursive(tp, hnb): split large tile tasks into sub-tasks of hnb
    (reference parsec_recursivecall, src/zpotrf_L.jdf:148-172, src/zgeqrf.jdf:126-509).  POTRF runs
    its diagonal tile, panel TRSM and trailing updates as sub-taskpools on hnb x hnb re-tilings
    (models/potrf.py).  GEQRF / GEQRF_PARAM taskpools are rebuilt in place as the tile engine with
    recursive task bodies: every GEQRT / TSQRT / UNMQR / TSMQR on hnb-wide column blocks of its tiles
    (models/qr.py _factor_rec; hnb rounded to a multiple of IB)."""
    tp.recursive_nb = int(hnb)
    build = getattr(tp, "_rec_build", None)
    if build is not None and 0 < int(hnb):
        new = build(int(hnb))
        keep = tp.name
        tp.__dict__.update(new.__dict__)
        tp.name = keep
    return 0


for _op in ("potrf", "geqrf"):
    register_op(_op + "_setrecursive", _setrecursive)


# Recursive-hint and synchronous variants of dplasma_z.h:68-83 (zpotrf_rec, zgeqrf_rec, zpoinv_sync,
# zgetrs_incpiv) and the per-precision band -> tridiagonal bulge chase (zhbrdt).
def potrf_rec(ctx, uplo, A, hmb):
    """dplasma_zpotrf_rec: Cholesky with the recursive-subtask hint (see _setrecursive)."""
    from .models import potrf as _pf
    tp = _pf.potrf_New(ctx, uplo, A)
    _setrecursive(tp, hmb)
    return tp.execute(ctx)


def geqrf_rec(ctx, A, T, hnb):
    """dplasma_zgeqrf_rec: QR with the recursive-subtask hint (see _setrecursive)."""
    tp = _qr.geqrf_New(ctx, A, T)
    _setrecursive(tp, hnb)
    tp.execute(ctx)
    return 0


def poinv_sync(ctx, uplo, A):
    """dplasma_zpoinv_sync: A := inv(A) as three blocking steps (potrf, trtri, lauum)."""
    from .models import potrf as _pf
    info = _pf.potrf(ctx, uplo, A)
    if info:
        return info
    _chol.trtri(ctx, uplo, dplasmaNonUnit, A)
    _chol.lauum(ctx, uplo, A)
    return 0


def getrs_incpiv(ctx, trans, A, L, IPIV, B):
    """dplasma_zgetrs_incpiv: solve after getrf_incpiv (NoTrans only, as in the reference)."""
    if trans != dplasmaNoTrans:
        raise ValueError("getrs_incpiv: only trans = NoTrans is supported (as in the reference)")
    _lui.trsmpl_incpiv(ctx, A, L, IPIV, B)
    _b3.trsm(ctx, dplasmaLeft, dplasmaUpper, dplasmaNoTrans, dplasmaNonUnit, 1.0, A, B)
    return 0


for _n, _f in (("potrf_rec", potrf_rec), ("geqrf_rec", geqrf_rec), ("poinv_sync", poinv_sync),
               ("getrs_incpiv", getrs_incpiv), ("hbrdt", _eig.hbrdt)):
    register_op(_n, _f)
