"""Scheduling knobs of the reference's dplasmaaux.c (src/dplasmaaux.c:59-111).

* :func:`get_priority_limit` -- ``{S,D,C,Z}<FUNCTION>`` environment variable (e.g. ``DPOTRF=8``):
  the reference's PRI_CHANGE, the number of final panels whose critical-path tasks lose their
  top priority (zpotrf_wrapper.c:201-203; zpotrf_L.jdf:116 priority expression).  dplasma_amd
  maps priority to the HIP stream a task is issued on: panels k < nt - PRI_CHANGE run on the
  high-priority panel stream, the last PRI_CHANGE panels on the normal-priority update stream.
* :func:`gemm_lookahead` -- dplasma_aux_getGEMMLookahead: one process -> no limit (every chunk
  may be in flight); several -> at least 2, enough for ~3 tiles per computational unit.  Here a
  computational unit is one GPU (its MFMA engine is fed one batched launch per chunk), and the
  look-ahead counts SUMMA k-chunks whose exchange may run ahead of the GEMM (models/gemm.py).
"""
from __future__ import annotations

import math
import os

import torch

_PREC_LETTER = {torch.float32: "S", torch.float64: "D", torch.complex64: "C", torch.complex128: "Z"}


def get_priority_limit(function: str, A) -> int:
    """Value of the environment variable <prec letter><function> (0 when unset or not numeric)."""
    if not function or A is None:
        return 0
    letter = _PREC_LETTER.get(getattr(A, "dtype", None))
    if letter is None:
        return 0
    v = os.environ.get(letter + function)
    try:
        return int(v) if v is not None else 0
    except ValueError:
        return 0


def gemm_lookahead(ctx, A) -> int:
    """Reference dplasma_aux_getGEMMLookahead adapted to one computational unit per GPU."""
    nodes = max(1, getattr(ctx, "world", 1))
    if nodes == 1:
        return max(A.mt, A.nt)
    alpha = 3.0 * nodes / max(1, A.mt * A.nt)
    return max(int(math.ceil(alpha)), 2)
