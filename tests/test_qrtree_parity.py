"""HQR elimination trees against the reference's closed-form index functions.

Oracle: the type / annihilator formulas of src/dplasma_hqr.c for the non-domino, non-tsrr trees --
hqr_gettype (:299-322), hqr_currpiv (:1241-1311), the flat and binary low-level trees
(hqr_low_flat_currpiv :327, hqr_low_binary_currpiv :389) and the flat / binary high-level trees
(hqr_high_flat_currpiv :912, hqr_high_binary_currpiv :952) -- written out here independently of
dplasma_amd/models/qrtree.py and compared row by row for a sweep of shapes (the reference's
pivgen tester, tests/TestsQRPivgen.cmake, checks the same functions for consistency)."""
import itertools

import pytest

from dplasma_amd.models import qrtree as q


def ref_type(k, m, a, p):
    if m < k + p:
        return 3
    return 1 if (m // p) % a == 0 else 0


def ref_low(kind, k, m, a, p):
    """Domain index of the annihilator of domain-head row m (flat / binary low-level trees)."""
    k_a = (k + p - 1 - m % p) // p // a
    if kind == q.FLAT_TREE:
        return k_a
    m_pa = (m // p) // a
    d = m_pa - k_a
    if d == 0:
        return 0
    t = 1
    while d % 2 == 0:
        d //= 2
        t *= 2
    return m_pa - t


def ref_high(kind, k, m):
    if kind == q.FLAT_TREE:
        return k
    d, t = m - k, 1
    if d == 0:
        return 0
    while d % 2 == 0:
        d //= 2
        t *= 2
    return m - t


def ref_currpiv(llvl, hlvl, k, m, a, p):
    rank = m % p
    tmpk = k // (p * a)
    ty = ref_type(k, m, a, p)
    if ty == 0:
        tmp = (m // p) // a
        return k + (m - k) % p if tmp == tmpk else tmp * a * p + rank
    if ty == 1:
        tmp = ref_low(llvl, k, m, a, p)
        return k + (m - k) % p if tmp == tmpk else tmp * a * p + rank
    return ref_high(hlvl, k, m)


@pytest.mark.parametrize("llvl,hlvl", list(itertools.product([q.FLAT_TREE, q.BINARY_TREE],
                                                             [q.FLAT_TREE, q.BINARY_TREE])))
def test_hqr_trees_match_reference_formulas(llvl, hlvl):
    n = 0
    for mt, nt, a, p in itertools.product([1, 5, 12, 23], [1, 4, 23], [1, 2, 3, 5], [1, 2, 3, 4]):
        t = q.HQRTree(mt, nt, llvl, hlvl, a, p)
        t.check()
        for k in range(min(mt, nt)):
            for m in range(k + 1, mt):
                ty = ref_type(k, m, q.HQRTree(mt, nt, llvl, hlvl, a, p).a, p)
                aa = t.a
                assert t.gettype(k, m) == ty, (mt, nt, a, p, k, m)
                assert t.currpiv(k, m) == ref_currpiv(llvl, hlvl, k, m, aa, p), (mt, nt, a, p, k, m, t.kills(k))
                n += 1
    assert n > 1000


@pytest.mark.parametrize("llvl", [q.FLAT_TREE, q.GREEDY_TREE, q.FIBONACCI_TREE, q.BINARY_TREE, q.GREEDY1P_TREE])
@pytest.mark.parametrize("hlvl", [q.FLAT_TREE, q.GREEDY_TREE, q.FIBONACCI_TREE, q.BINARY_TREE])
def test_hqr_every_tree_valid(llvl, hlvl):
    """Every tree combination is a valid elimination plan (dplasma_qrtree_check) whose TS domains
    are the globally aligned groups of a local rows and whose pivots sit above their victims."""
    for mt, nt, a, p in itertools.product([3, 11, 30], [2, 11, 30], [1, 2, 4], [1, 2, 3]):
        t = q.HQRTree(mt, nt, llvl, hlvl, a, p)
        t.check()
        for k in range(min(mt, nt)):
            for (pv, m, ty) in t.kills(k):
                assert pv < m
                if ty == q.KILLED_BY_TS:
                    assert pv % p == m % p          # TS kills stay inside a process row
                    assert (m // p) // t.a == (pv // p) // t.a or pv < k + p
