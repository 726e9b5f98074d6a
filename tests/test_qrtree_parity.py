"""Every QR reduction tree against the reference's own tree code.

tests/fixtures/qrtree_ref.json holds the digest of each tree of the sweep below as computed by the
reference's dplasma_hqr.c / dplasma_systolic_qr.c compiled into an oracle
(tools/qrtree_oracle/build.sh, oracle.c; regenerate with ``compare.py --write``).  The digest covers,
per panel k: the GEQRT rows in getm order and, per row, gettype, currpiv and the complete nextpiv and
prevpiv chains -- so a tree passes only if every query answers exactly what the reference answers.
Sweep: tests/TestsQRPivgen.cmake:140-206 style -- HQR (llvl 0-4, hlvl 0-4, a in {1,2,4},
p in {1,3,5}, domino, tsrr, M in {1,3,4,10,17,25}, N in {1,2,5,13}), the adaptive SVD tree
(hlvl 0-4, p 1-3, cores, ratio) and the systolic tree.
"""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools", "qrtree_oracle"))

import compare  # noqa: E402

from dplasma_amd.models import qrtree as Q  # noqa: E402

REF = json.load(open(os.path.join(ROOT, "tests", "fixtures", "qrtree_ref.json")))["trees"]


def _sweep(kind):
    return [c for c in compare.configs() if c[0] == kind and compare.key(c) in REF]


@pytest.mark.parametrize("kind,llvl", [("hqr", l) for l in range(5)] + [("svd", None), ("sys", None)])
def test_tree_matches_reference(kind, llvl):
    cfgs = [c for c in _sweep(kind) if llvl is None or c[3] == llvl]
    assert len(cfgs) > 50
    bad = [compare.key(c) for c in cfgs if compare.digest(compare.ours(c)) != REF[compare.key(c)]]
    assert not bad, f"{len(bad)}/{len(cfgs)} trees differ from the reference, e.g. {bad[:5]}"


@pytest.mark.parametrize("cfg", ["hqr 25 13 4 2 2 3 1 1", "hqr 17 5 1 3 4 5 0 1", "svd 25 13 0 3 2 1",
                                 "sys 25 13 4 2"])
def test_plans_valid(cfg):
    """The elimination plans derived from the queries are valid programs (every row killed once,
    after its own kills; TS only onto triangles; currpiv agrees)."""
    c = cfg.split()
    kind, args = c[0], list(map(int, c[1:]))
    if kind == "hqr":
        t = Q.HQRTree(*args)
    elif kind == "svd":
        t = Q.SVDTree(*args)
    else:
        t = Q.SystolicTree(*args)
    t.check()
    for k in range(min(t.mt, t.nt)):
        assert sorted(m for _, m, _ in t.kills(k)) == list(range(k + 1, t.mt))
