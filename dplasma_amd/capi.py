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
