"""The C++ reduction trees of the interpreter-free engine (capi/native_qrtree.cpp) against the reference.

Each tree of the parity sweep (tools/qrtree_oracle/compare.py configs: HQR llvl 0-4 x hlvl 0-4 x a x p x
domino x tsrr, the adaptive SVD tree, the systolic tree) is built in C++ through the test hooks
dpl_nq_create / dpl_nq_query of libdplasma.so, canonicalised exactly like the Python trees (every query:
getm, gettype, currpiv, the complete nextpiv / prevpiv chains) and its digest compared with the digest of
the reference's own dplasma_hqr.c / dplasma_systolic_qr.c in tests/fixtures/qrtree_ref.json.  No GPU."""
import ctypes
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools", "qrtree_oracle"))

import compare  # noqa: E402

LIB = os.path.join(ROOT, "dplasma_amd", "lib", "libdplasma.so")
REF = json.load(open(os.path.join(ROOT, "tests", "fixtures", "qrtree_ref.json")))["trees"]


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.skip("libdplasma.so not built (python tools/build.py)")
    L = ctypes.CDLL(LIB)
    L.dpl_nq_create.restype = ctypes.c_void_p
    L.dpl_nq_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    L.dpl_nq_query.restype = ctypes.c_int
    L.dpl_nq_query.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    L.dpl_nq_free.argtypes = [ctypes.c_void_p]
    return L


class _CTree:
    """The query interface of one C++ tree (what compare.canon walks)."""

    def __init__(self, L, cfg):
        self.L = L
        kind, m, n = cfg[0], cfg[1], cfg[2]
        if kind == "hqr":
            code, args = 0, list(cfg[3:])
        elif kind == "svd":
            code, args = 2, list(cfg[3:]) + [cfg[4]]     # nodes = p (models/qrtree.py SVDTree default)
        else:
            code, args = 1, list(cfg[3:])
        arr = (ctypes.c_int * 8)(*args)
        self.h = L.dpl_nq_create(code, m, n, arr)
        assert self.h

    def close(self):
        self.L.dpl_nq_free(self.h)

    def q(self, fn, k, x=0, y=0):
        return self.L.dpl_nq_query(self.h, fn, k, x, y)

    def getnbgeqrf(self, k):
        return self.q(0, k)

    def getm(self, k, i):
        return self.q(1, k, i)

    def gettype(self, k, m):
        return self.q(2, k, m)

    def currpiv(self, k, m):
        return self.q(3, k, m)

    def nextpiv(self, k, p, s):
        return self.q(4, k, p, s)

    def prevpiv(self, k, p, s):
        return self.q(5, k, p, s)

    def check(self):
        return self.q(6, 0)


def _sweep(kind):
    return [c for c in compare.configs() if c[0] == kind and compare.key(c) in REF]


@pytest.mark.parametrize("kind,llvl", [("hqr", l) for l in range(5)] + [("svd", None), ("sys", None)])
def test_native_tree_matches_reference(lib, kind, llvl):
    cfgs = [c for c in _sweep(kind) if llvl is None or c[3] == llvl]
    assert len(cfgs) > 50
    bad = []
    for c in cfgs:
        t = _CTree(lib, c)
        try:
            if compare.digest(compare.canon(t, c[1], c[2])) != REF[compare.key(c)]:
                bad.append(compare.key(c))
        finally:
            t.close()
    assert not bad, f"{len(bad)}/{len(cfgs)} C++ trees differ from the reference, e.g. {bad[:5]}"


@pytest.mark.parametrize("cfg", ["hqr 25 13 4 2 2 3 1 1", "hqr 17 5 1 3 4 5 0 1", "hqr 40 40 1 0 4 1 0 0",
                                 "svd 25 13 0 3 2 1", "sys 25 13 4 2"])
def test_native_plans_valid(lib, cfg):
    """The C++ plan validation (Tree::check: every row killed once, after its own kills; TS only onto
    triangles; currpiv agrees with the plan) passes on representative trees."""
    c = cfg.split()
    t = _CTree(lib, [c[0]] + list(map(int, c[1:])))
    try:
        assert t.check() == 0
    finally:
        t.close()
