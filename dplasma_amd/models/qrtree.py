"""Reduction trees for hierarchical tile QR/LQ (pure integer logic).

Reference: ``src/include/dplasma/qr_param.h:18-148`` (the ``dplasma_qrtree_t``
query interface), ``src/dplasma_hqr.c`` (3-level HQR trees), ``src/dplasma_systolic_qr.c``
(systolic 2-level tree) and ``src/dplasma_hqr_dbg.c`` (validation / printers).

Design: a tree answers the reference's query interface (getnbgeqrf, getm, geti, gettype,
currpiv, nextpiv, prevpiv) with the reference's own semantics -- the index functions of
``dplasma_hqr.c`` (HQR and the adaptive SVD tree) and ``dplasma_systolic_qr.c``, pinned tree by tree
to the reference code compiled as an oracle (tools/qrtree_oracle, tests/test_qrtree_parity.py:
every tree of the reference's pivgen sweep shape identical, chains and all).  From the queries each
tree derives an explicit *elimination plan* per panel k for the tile-DAG runtime:

* ``heads(k)``  -- the rows that get a GEQRT at step k (getm),
* ``kills(k)``  -- ordered list of ``(piv, m, type)``: row m annihilated by row piv with a TS
  kernel (type 0) or a TT kernel (1 local tree, 2 domino, 3 distributed tree), every annihilator's
  kills in its nextpiv order and every row's own kills before it is killed (post-order of the
  elimination tree).

``runtime/dag.py`` turns the plan into a leveled DAG, so all eliminations of one tree round land in
the same batched launch.

Tree shapes over an ordered row list (element 0 is the survivor):
  FLAT       sequential: r0 kills r1, r2, ...
  GREEDY     each round the bottom half is killed by the top half (log depth)
  FIBONACCI  each round kills a Fibonacci-limited number of bottom rows
  BINARY     pairwise at doubling distance (r0<-r1, r2<-r3; r0<-r2; ...)
  GREEDY1P   greedy that keeps one annihilator per round and process row group
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence, Tuple

from ..constants import dplasmaNoTrans

FLAT_TREE, GREEDY_TREE, FIBONACCI_TREE, BINARY_TREE, GREEDY1P_TREE = 0, 1, 2, 3, 4
KILLED_BY_TS, KILLED_BY_LOCALTREE, KILLED_BY_DOMINO, KILLED_BY_DISTTREE = 0, 1, 2, 3
TREE_NAMES = {FLAT_TREE: "flat", GREEDY_TREE: "greedy", FIBONACCI_TREE: "fibonacci", BINARY_TREE: "binary",
              GREEDY1P_TREE: "greedy1p"}


def tree_pairs(rows: Sequence[int], tree: int) -> List[Tuple[int, int]]:
    """Elimination pairs (piv, victim) reducing ``rows`` to rows[0], in a valid order."""
    rows = list(rows)
    if len(rows) <= 1:
        return []
    out = []
    if tree == FLAT_TREE:
        return [(rows[0], r) for r in rows[1:]]
    if tree == BINARY_TREE:
        d = 1
        while d < len(rows):
            for i in range(0, len(rows), 2 * d):
                if i + d < len(rows):
                    out.append((rows[i], rows[i + d]))
            d *= 2
        return out
    if tree in (GREEDY_TREE, GREEDY1P_TREE):
        alive = rows
        while len(alive) > 1:
            h = len(alive) // 2
            if tree == GREEDY1P_TREE and len(alive) > 2:
                h = max(1, h - 1) if len(alive) % 2 == 0 else h
            piv, vic = alive[:len(alive) - h], alive[len(alive) - h:]
            out += [(piv[i], vic[i]) for i in range(h)]
            alive = piv
        return out
    if tree == FIBONACCI_TREE:
        fib = [1, 1]
        while fib[-1] < len(rows):
            fib.append(fib[-1] + fib[-2])
        alive = rows
        while len(alive) > 1:
            h = max(f for f in fib if f <= len(alive) // 2)
            piv, vic = alive[:len(alive) - h], alive[len(alive) - h:]
            out += [(piv[i], vic[i]) for i in range(h)]
            alive = piv
        return out
    raise ValueError(f"unknown tree type {tree}")


class QRTree:
    """A reduction tree: reference query interface + the elimination plans derived from it.

    ``mt``/``nt``: tile rows/cols of the (logical) matrix being factored (for an LQ tree built with
    trans=ConjTrans these are A.nt / A.mt).  Subclasses implement getnbgeqrf, getm, gettype,
    currpiv, nextpiv, prevpiv."""

    def __init__(self, mt: int, nt: int, a: int, p: int, name: str):
        self.mt, self.nt, self.a, self.p = mt, nt, a, p
        self.name = name
        self._plans: Dict[int, Tuple[List[int], List[Tuple[int, int, int]]]] = {}

    # ------------------------------------------------------------ plans (derived from the queries)
    def _plan(self, k: int):
        pl = self._plans.get(k)
        if pl is not None:
            return pl
        mt = self.mt
        heads = [self.getm(k, i) for i in range(self.getnbgeqrf(k))]
        kills: List[Tuple[int, int, int]] = []
        # post-order over the elimination tree rooted at the diagonal row: a row's own kills (in
        # its nextpiv order) come before the kill that eliminates it
        stack = [(k, self.nextpiv(k, k, mt))]
        while stack:
            piv, nxt = stack[-1]
            if nxt == mt:
                stack.pop()
                if stack:
                    parent, m = stack[-1]
                    kills.append((parent, piv, self.gettype(k, piv)))
                    stack[-1] = (parent, self.nextpiv(k, parent, piv))
                continue
            stack.append((nxt, self.nextpiv(k, nxt, mt)))
        pl = self._plans[k] = (heads, kills)
        return pl

    def heads(self, k: int) -> List[int]:
        return self._plan(k)[0]

    def kills(self, k: int) -> List[Tuple[int, int, int]]:
        return self._plan(k)[1]

    def geti(self, k: int, m: int) -> int:
        return self.heads(k).index(m)

    # ------------------------------------------------------------ validation / debug
    def check(self) -> int:
        """Validate the plans (dplasma_qrtree_check analogue): 0 if valid, else raises."""
        for k in range(min(self.mt, self.nt)):
            heads = set(self.heads(k))
            if k not in heads:
                raise AssertionError(f"panel {k}: diagonal row is not a GEQRT head")
            killed = set()
            alive = set(range(k, self.mt))
            for (p, m, t) in self.kills(k):
                if not (k <= p < self.mt and k < m < self.mt):
                    raise AssertionError(f"panel {k}: bad pair ({p}, {m})")
                if m in killed or p in killed:
                    raise AssertionError(f"panel {k}: row used after being killed ({p}, {m})")
                if t == KILLED_BY_TS and m in heads:
                    raise AssertionError(f"panel {k}: TS kill of a GEQRT row {m}")
                if t != KILLED_BY_TS and (m not in heads or p not in heads):
                    raise AssertionError(f"panel {k}: TT kill between non-triangular rows ({p}, {m})")
                if t == KILLED_BY_TS and p not in heads:
                    raise AssertionError(f"panel {k}: TS annihilator {p} is not triangular")
                if self.currpiv(k, m) != p:
                    raise AssertionError(f"panel {k}: currpiv({m}) = {self.currpiv(k, m)} != {p}")
                killed.add(m)
            if alive - killed != {k}:
                raise AssertionError(f"panel {k}: survivors {sorted(alive - killed)} != [{k}]")
            for m in range(k + 1, self.mt):
                if m not in heads and self.gettype(k, m) != KILLED_BY_TS:
                    raise AssertionError(f"panel {k}: row {m} neither GEQRT'ed nor TS-killed")
        return 0

    def depth(self, k: int) -> int:
        """Critical path (rounds) of panel k's elimination (TS kills count 1 each along a chain)."""
        t = {m: 0 for m in range(k, self.mt)}
        for (p, m, _) in self.kills(k):
            d = max(t[p], t[m]) + 1
            t[p] = t[m] = d
        return max(t.values()) if t else 0

    def print_type(self) -> str:
        lines = []
        for m in range(self.mt):
            lines.append(" ".join(("%2d" % self.gettype(k, m)) if m >= k else " ." for k in range(min(self.mt, self.nt))))
        return "\n".join(lines)

    def print_pivot(self) -> str:
        lines = []
        for m in range(self.mt):
            lines.append(" ".join(("%3d" % self.currpiv(k, m)) if m > k else "  ." for k in range(min(self.mt, self.nt))))
        return "\n".join(lines)

    def print_nbgeqrt(self) -> str:
        return " ".join(str(self.getnbgeqrf(k)) for k in range(min(self.mt, self.nt)))

    def dot(self, k: int = None) -> str:
        """DOT graph of the eliminations (dplasma_qrtree_print_dag analogue)."""
        ks = range(min(self.mt, self.nt)) if k is None else [k]
        out = ["digraph qrtree {"]
        for kk in ks:
            for (p, m, t) in self.kills(kk):
                style = "solid" if t else "dashed"
                out.append(f'  "k{kk}_{m}" -> "k{kk}_{p}" [style={style},label="{t}"];')
        out.append("}")
        return "\n".join(out)

    def __repr__(self):
        return f"QRTree({self.name}, mt={self.mt}, nt={self.nt}, a={self.a}, p={self.p})"


# ----------------------------------------------------------------------------- sub-trees
# The two reduction levels of the hierarchical tree (dplasma_hqr.c:100-1240): a "low" tree reducing
# the domain heads of one process row (indices are domain indices, ldd of them) and a "high" tree
# reducing the p rows of the distributed band (global row indices, ldd = mt).  Each answers currpiv /
# nextpiv / prevpiv; nextpiv(start = ldd) is the first victim, prevpiv(start = the pivot) the last.
def _c_mod(a: int, b: int) -> int:
    """C's remainder (truncating division) for the reference's formulas with negative operands."""
    r = abs(a) % abs(b)
    return -r if a < 0 else r


def _nbextra1(k: int, pa: int, p: int) -> int:
    return _c_mod(-k, pa) + pa if (k % pa) > (pa - p) else 0


def _ilog2_floor(x: int) -> int:
    return int(math.log(x) / math.log(2.0)) if x > 0 else -1


class _Sub:
    def __init__(self, ldd: int, a: int, p: int, domino: bool, min_mn: int):
        self.ldd, self.a, self.p, self.domino, self.min_mn = ldd, a, p, domino, min_mn

    def k_a(self, k: int, row: int) -> int:
        return k // self.a if self.domino else (k + self.p - 1 - row % self.p) // self.p // self.a


class _LowFlat(_Sub):
    def currpiv(self, k, m):
        return self.k_a(k, m)

    def nextpiv(self, k, p, s):
        ka, ppa = self.k_a(k, p), (p // self.p) // self.a
        if s <= ppa:
            return self.ldd
        if ppa == ka and self.ldd - ka > 1:
            if s == self.ldd:
                return ppa + 1
            if s < self.ldd:
                return s + 1
        return self.ldd

    def prevpiv(self, k, p, s):
        ka, ppa = self.k_a(k, p), (p // self.p) // self.a
        if ppa == ka and self.ldd - ka > 1:
            if s == ppa:
                return self.ldd - 1
            if s > ppa + 1:
                return s - 1
        return self.ldd


def _binary_currpiv(off_m: int, base: int) -> int:
    if off_m == 0:
        return 0
    step = off_m & -off_m
    return base + off_m - step


class _LowBinary(_Sub):
    def currpiv(self, k, m):
        ka, mpa = self.k_a(k, m), (m // self.p) // self.a
        d = mpa - ka
        return 0 if d == 0 else mpa - (d & -d)

    def nextpiv(self, k, p, s):
        ka, ppa = self.k_a(k, p), (p // self.p) // self.a
        if s <= ppa:
            return self.ldd
        off, bit = ppa - ka, 0
        if s != self.ldd:
            while ((s - ka) & (1 << bit)) == 0:
                bit += 1
            bit += 1
        t = off | (1 << bit)
        return t + ka if t != off and t + ka < self.ldd else self.ldd

    def prevpiv(self, k, p, s):
        ka, ppa = self.k_a(k, p), (p // self.p) // self.a
        off = ppa - ka
        if s == ppa and off % 2 == 0:
            if off == 0:
                bit = _ilog2_floor(self.ldd - ka)
            else:
                bit = 0
                while (off & (1 << bit)) == 0:
                    bit += 1
            for i in range(bit, -1, -1):
                t = off | (1 << i)
                if off != t and t + ka < self.ldd:
                    return t + ka
            return self.ldd
        if s - ppa > 1:
            return ppa + ((s - ppa) >> 1)
        return self.ldd


class _LowTable(_Sub):
    """Low trees given by a pivot table ipiv[section][k][domain] (fibonacci, greedy, greedy1p):
    nextpiv scans downwards from start-1, prevpiv upwards from start+1."""

    def _col(self, k, row):
        raise NotImplementedError

    def currpiv(self, k, m):
        return self._col(k, m)[(m // self.p) // self.a]

    def nextpiv(self, k, p, s):
        col, ka = self._col(k, p), self.k_a(k, p)
        ppa = self._ppa(p)
        for i in range(s - 1, ka, -1):
            if col[i] == ppa:
                return i
        return self.ldd

    def prevpiv(self, k, p, s):
        col = self._col(k, p)
        ppa = (p // self.p) // self.a
        for i in range(s + 1, self.ldd):
            if col[i] == ppa:
                return i
        return self.ldd

    def _ppa(self, p):
        return (p // self.p) // self.a


class _LowFib(_LowTable):
    def __init__(self, *args):
        super().__init__(*args)
        mt = self.ldd
        self.tab = [[0] * mt for _ in range(self.min_mn)]
        f1, m = 1, 1
        while m < mt:
            kk = 0
            while kk < f1 and m < mt:
                self.tab[0][m] = m - f1
                kk, m = kk + 1, m + 1
            f1 += 1
        for k in range(1, self.min_mn):
            for m in range(k + 1, mt):
                self.tab[k][m] = self.tab[k - 1][m - 1] + 1

    def _col(self, k, row):
        return self.tab[self.k_a(k, row)]


class _LowGreedy(_LowTable):
    """Coarse-grained greedy (dplasma_hqr.c:584-716): per panel, half of the domains still to be
    annihilated are killed by those just above them; a column starts a round as soon as its
    predecessor has produced enough triangles."""

    def __init__(self, *args):
        super().__init__(*args)
        mt, a, p = self.ldd, self.a, self.p
        pa = p * a
        if self.domino:
            self.min_mn = min(self.min_mn, mt * a)
            mn = self.min_mn
            tab = [[0] * mt for _ in range(mn)]
            nT, nZ = [0] * mn, [0] * mn
            nT[0] = mt
            k = first = 0
            while not (nT[mn - 1] == mt - (mn - 1) // a and nZ[mn - 1] + 1 == nT[mn - 1]) and first < mn:
                h = (nT[k] - nZ[k]) // 2
                if h == 0:
                    while first < mn and nT[first] == mt - first // a and nZ[first] + 1 == nT[first]:
                        if first % a != a - 1 and first < mn - 1:
                            nT[first + 1] += 1
                        first += 1
                    k = first
                    continue
                if k < mn - 1:
                    nT[k + 1] += h
                top = mt - nZ[k] - 1
                nZ[k] += h
                for j in range(top, top - h, -1):
                    tab[k][j] = j - h
                k += 1
                if k > mn - 1:
                    k = first
            self.tab = [tab]
        else:
            mn = self.min_mn
            self.tab = []
            for r in range(p):
                tab = [[0] * mt for _ in range(mn)]
                lmn = mn
                todo = [0] * mn
                for k in range(mn):
                    todo[k] = max(mt - (k + p - 1 - r) // pa, 0)
                    if todo[k] == 0:
                        lmn = k
                        break
                nT, nZ = [0] * mn, [0] * mn
                nT[0] = mt
                k = first = 0
                while lmn > 0 and not (nT[lmn - 1] == todo[lmn - 1] and nZ[lmn - 1] + 1 == nT[lmn - 1]) \
                        and first < lmn:
                    h = (nT[k] - nZ[k]) // 2
                    if h == 0:
                        while first < lmn and nT[first] == todo[first] and nZ[first] + 1 == nT[first]:
                            if first < lmn - 1 and first % pa != (a - 1) * p + r:
                                nT[first + 1] += 1
                            first += 1
                        k = first
                        continue
                    if k < lmn - 1:
                        nT[k + 1] += h
                    top = mt - nZ[k] - 1
                    nZ[k] += h
                    for j in range(top, top - h, -1):
                        tab[k][j] = j - h
                    k += 1
                    if k > lmn - 1:
                        k = first
                self.tab.append(tab)

    def _col(self, k, row):
        return self.tab[0 if self.domino else row % self.p][k]

    def _ppa(self, p):
        return p // (self.p * self.a)


class _LowGreedy1p(_LowGreedy):
    """Per-panel greedy (dplasma_hqr.c:789-910): every column reduced independently by halving."""

    def __init__(self, ldd, a, p, domino, min_mn):
        _Sub.__init__(self, ldd, a, p, domino, min_mn)
        mt, pa = ldd, p * a

        def halve(col, nT):
            nZ = 0
            while nZ < nT - 1:
                h = (nT - nZ) // 2
                top = mt - nZ - 1
                nZ += h
                for j in range(top, top - h, -1):
                    col[j] = j - h
        if domino:
            self.min_mn = min(min_mn, mt * a)
            tab = [[0] * mt for _ in range(self.min_mn)]
            for k in range(self.min_mn):
                halve(tab[k], max(mt - k // a, 0))
            self.tab = [tab]
        else:
            self.tab = []
            for r in range(p):
                tab = [[0] * mt for _ in range(min_mn)]
                for k in range(min_mn):
                    nT = max(mt - (k + p - 1 - r) // pa, 0)
                    if nT == 0:
                        break
                    halve(tab[k], nT)
                self.tab.append(tab)


class _HighFlat(_Sub):
    def currpiv(self, k, m):
        return k

    def nextpiv(self, k, p, s):
        if p == k and self.ldd > 1:
            if s == self.ldd:
                return p + 1
            if s < self.ldd and s - k < self.p - 1:
                return s + 1
        return self.ldd

    def prevpiv(self, k, p, s):
        if p == k and self.ldd > 1:
            if s == p and p != self.ldd - 1:
                return min(p + self.p - 1, self.ldd - 1)
            if s > p + 1 and s - k < self.p:
                return s - 1
        return self.ldd


class _HighBinary(_Sub):
    def currpiv(self, k, m):
        d = m - k
        return 0 if d == 0 else m - (d & -d)

    def nextpiv(self, k, p, s):
        if s <= p:
            return self.ldd
        off, bit = p - k, 0
        if s != self.ldd:
            while ((s - k) & (1 << bit)) == 0:
                bit += 1
            bit += 1
        t = off | (1 << bit)
        return t + k if t != off and t < self.p and t + k < self.ldd else self.ldd

    def prevpiv(self, k, p, s):
        off = p - k
        if s == p and off % 2 == 0:
            if off == 0:
                bit = _ilog2_floor(min(self.p, self.ldd - k))
            else:
                bit = 0
                while (off & (1 << bit)) == 0:
                    bit += 1
            for i in range(bit, -1, -1):
                t = off | (1 << i)
                if off != t and t < self.p and t + k < self.ldd:
                    return t + k
            return self.ldd
        if s - p > 1:
            return p + ((s - p) >> 1)
        return self.ldd


class _HighFib(_Sub):
    """Fibonacci band tree (one pivot vector for every panel); also the greedy1p band tree, whose
    vector is the greedy reduction of the first panel (dplasma_hqr.c:1062-1145)."""

    def __init__(self, ldd, a, p, domino, min_mn, greedy1p=False):
        super().__init__(ldd, a, p, domino, min_mn)
        self.tab = [0] * p
        if greedy1p:
            mt = ldd
            nT, nZ = mt, max(mt - p, 0)
            while not (nT == mt and nZ + 1 == nT):
                h = (nT - nZ) // 2
                if h == 0:
                    break
                top = mt - nZ - 1
                nZ += h
                for j in range(top, top - h, -1):
                    self.tab[j] = j - h
        else:
            f1, m = 1, 1
            while m < p:
                kk = 0
                while kk < f1 and m < p:
                    self.tab[m] = m - f1
                    kk, m = kk + 1, m + 1
                f1 += 1

    def currpiv(self, k, m):
        return self.tab[m - k] + k

    def nextpiv(self, k, p, s):
        for i in range(min(s - k - 1, self.p - 1), 0, -1):
            if self.tab[i] == p - k:
                return i + k
        return self.ldd

    def prevpiv(self, k, p, s):
        lp, end = p - k, min(self.ldd - k, self.p)
        for i in range(s - k + 1, end):
            if self.tab[i] == lp:
                return i + k
        return self.ldd


class _HighGreedy(_Sub):
    def __init__(self, *args):
        super().__init__(*args)
        mt, p, mn = self.ldd, self.p, self.min_mn
        self.tab = [[0] * p for _ in range(mn)]
        nT, nZ = [0] * mn, [0] * mn
        nT[0], nZ[0] = mt, max(mt - p, 0)
        for k in range(1, mn):
            nT[k] = nZ[k] = max(mt - k - p, 0)
        k = first = 0
        while not (nT[mn - 1] == mt - (mn - 1) and nZ[mn - 1] + 1 == nT[mn - 1]) and first < mn:
            h = (nT[k] - nZ[k]) // 2
            if h == 0:
                while first < mn and nT[first] == mt - first and nZ[first] + 1 == nT[first]:
                    first += 1
                k = first
                continue
            top = mt - nZ[k] - 1
            nZ[k] += h
            if k < mn - 1:
                nT[k + 1] = nZ[k]
            for j in range(top, top - h, -1):
                self.tab[k][j - k] = j - h
            k += 1
            if k > mn - 1:
                k = first

    def currpiv(self, k, m):
        return self.tab[k][m - k]

    def nextpiv(self, k, p, s):
        for i in range(min(s - 1, k + self.p - 1), k, -1):
            if self.tab[k][i - k] == p:
                return i
        return self.ldd

    def prevpiv(self, k, p, s):
        for i in range(s - k + 1, self.p):
            if self.tab[k][i] == p:
                return k + i
        return self.ldd


def _low_tree(kind, ldd, a, p, domino, min_mn):
    cls = {FLAT_TREE: _LowFlat, FIBONACCI_TREE: _LowFib, BINARY_TREE: _LowBinary, GREEDY1P_TREE: _LowGreedy1p}
    return cls.get(kind, _LowGreedy)(ldd, a, p, domino, min_mn)


def _high_tree(kind, mt, a, p, domino, min_mn, default_flat=True):
    if kind == FLAT_TREE:
        return _HighFlat(mt, a, p, domino, min_mn)
    if kind == GREEDY_TREE:
        return _HighGreedy(mt, a, p, domino, min_mn)
    if kind == GREEDY1P_TREE:
        return _HighFib(mt, a, p, domino, min_mn, greedy1p=True)
    if kind == BINARY_TREE:
        return _HighBinary(mt, a, p, domino, min_mn)
    if kind == FIBONACCI_TREE or not default_flat:
        return _HighFib(mt, a, p, domino, min_mn)
    return _HighFlat(mt, a, p, domino, min_mn)


class HQRTree(QRTree):
    """Hierarchical tree (dplasma_hqr_init, src/dplasma_hqr.c:1790-1945), reference semantics:
    TS domains of ``a`` local rows (flat TS chains), a low-level tree ``llvl`` over the domain heads
    of each of the ``p`` process rows, a high-level tree ``hlvl`` over the p-row distributed band;
    ``domino`` couples consecutive panels with type-2 TT kills, ``tsrr`` rotates the TS killers of
    every domain group round-robin per panel (the row permutation of hqr_genperm).  Query functions:
    dplasma_hqr.c:182-322 (getnbgeqrf, getm, geti, gettype), 1241-1568 (currpiv, nextpiv, prevpiv)."""

    def __init__(self, mt, nt, llvl=GREEDY_TREE, hlvl=FLAT_TREE, a=1, p=1, domino=False, tsrr=False):
        self.llvl, self.hlvl = llvl, hlvl
        a = 4 if a == -1 else max(a, 1)
        p = max(p, 1)
        ratio = nt / mt if mt else 1.0
        if isinstance(domino, bool) or domino >= 0:
            domino = bool(domino)
        else:
            domino = ratio < 0.5
        self.domino, self.tsrr = domino, bool(tsrr)
        a = min(a, mt)
        super().__init__(mt, nt, a, p, "hqr")
        min_mn = min(mt, nt)
        low_mt = (mt + p * a - 1) // (p * a)
        self._low = _low_tree(llvl, low_mt, a, p, domino, min_mn)
        self._high = _high_tree(hlvl, mt, a, p, domino, min_mn, default_flat=ratio >= 0.5) if p > 1 else None
        self._genperm()

    # ---- tsrr permutation (hqr_genperm, dplasma_hqr.c:1570-1640)
    def _genperm(self):
        m, n, a, p = self.mt, self.nt, self.a, self.p
        pa = p * a
        endpa = m - m % pa
        self._perm = []
        self._inv = []
        for k in range(min(m, n)):
            if not self.tsrr:
                perm = list(range(m + 1))
            else:
                perm = [-1] * (m + 1)
                end2 = p + (k * p if self.domino else k + _nbextra1(k, pa, p))
                end2 = min((end2 + pa - 1) // pa * pa, m)
                i = k
                for i in range(k, end2):
                    perm[i] = i
                i = max(end2, k)
                while i < endpa:
                    for j in range(pa):
                        perm[i + j] = i + (j + p * (k % a)) % pa
                    i += pa
                for i in range(i, m):
                    perm[i] = i
                perm[m] = m
            inv = {v: i for i, v in enumerate(perm) if v >= 0}
            self._perm.append(perm)
            self._inv.append(inv)

    def _invperm(self, k, m):
        return m if self.a == 1 else self._inv[k].get(m, m)

    # ---- reference query interface
    def getnbgeqrf(self, k):
        a, p, gmt = self.a, self.p, self.mt
        pa = p * a
        if self.domino:
            nb2 = k * (p - 1)
            nb11 = (p * (k + 1) + pa - 1) // pa * pa
        else:
            nb2 = _nbextra1(k, pa, p)
            nb11 = (k + p + pa - 1) // pa * pa
        nb12 = (gmt // pa) * pa
        nb1 = (nb12 - nb11) // a + min(p, gmt - nb12)   # C truncation: nb12 >= nb11 - pa here
        if nb12 - nb11 < 0:
            nb1 = int((nb12 - nb11) / a) + min(p, gmt - nb12)
        return min(nb1 + nb2 + p, gmt - k)

    def getm(self, k, i):
        a, p = self.a, self.p
        pa = p * a
        nb23 = p + (k * (p - 1) if self.domino else _nbextra1(k, pa, p))
        if i < nb23:
            return k + i
        j = i - nb23
        pos1 = ((p * (k + 1) if self.domino else p + k) + pa - 1) // pa * pa
        return self._perm[k][pos1 + (j // p) * pa + j % p]

    def gettype(self, k, m):
        a, p = self.a, self.p
        lm = self._invperm(k, m)
        if lm < k + p:
            return KILLED_BY_DISTTREE
        if self.domino and lm < p * (k + 1):
            return KILLED_BY_DOMINO
        return KILLED_BY_LOCALTREE if (lm // p) % a == 0 else KILLED_BY_TS

    def currpiv(self, k, m):
        a, p, gmt = self.a, self.p, self.mt
        pm = self._invperm(k, m)
        lm, rank = pm // p, pm % p
        perm = self._perm[k]
        t = self.gettype(k, m)
        if self.domino:
            if t == KILLED_BY_TS:
                tmp = lm // a
                return perm[k * p + rank] if tmp == k // a else perm[tmp * a * p + rank]
            if t == KILLED_BY_LOCALTREE:
                tmp = self._low.currpiv(k, pm)
                return perm[k * p + rank if tmp == k // a else tmp * a * p + rank]
            if t == KILLED_BY_DOMINO:
                return m - p
            return self._high.currpiv(k, pm) if self._high is not None else gmt
        tmpk = k // (p * a)
        if t == KILLED_BY_TS:
            tmp = lm // a
            return perm[k + (pm - k) % p if tmp == tmpk else tmp * a * p + rank]
        if t == KILLED_BY_LOCALTREE:
            tmp = self._low.currpiv(k, pm)
            return perm[k + (pm - k) % p if tmp == tmpk else tmp * a * p + rank]
        if t == KILLED_BY_DOMINO:
            return perm[pm - p]
        return perm[self._high.currpiv(k, pm)] if self._high is not None else gmt

    def nextpiv(self, k, pivot, start):
        a, p, gmt = self.a, self.p, self.mt
        low = self._low
        ostart, opivot = start, pivot
        start = self._invperm(k, ostart) if ostart != gmt else gmt
        pivot = self._invperm(k, opivot)
        lpivot, rpivot = pivot // p, pivot % p
        lstart = low.ldd * a if start == gmt else start // p
        perm = self._perm[k]
        ls = self.gettype(k, ostart) if start < gmt else -1
        lp = self.gettype(k, opivot)
        stage = ls
        if stage == -1:
            if lp == KILLED_BY_TS:
                return gmt
            stage = KILLED_BY_TS
        if stage == KILLED_BY_TS:
            if not (self.domino and lpivot < k):
                nextp = pivot + p if start == gmt else start + p
                if nextp < gmt and nextp < pivot + a * p and (nextp // p) % a != 0:
                    return perm[nextp]
                start, lstart = gmt, low.ldd * a
                stage = KILLED_BY_LOCALTREE
            else:
                stage = KILLED_BY_DOMINO
                start, lstart = gmt, low.ldd * a
        if stage == KILLED_BY_LOCALTREE:
            if not (self.domino and lpivot < k):
                tmp = low.nextpiv(k, pivot, lstart // a)
                if tmp * a * p + rpivot >= gmt and tmp == low.ldd - 1:
                    tmp = low.nextpiv(k, pivot, tmp)
                if tmp != low.ldd:
                    return perm[tmp * a * p + rpivot]
            start, lstart = gmt, low.ldd * a
            stage = KILLED_BY_DOMINO
        if stage == KILLED_BY_DOMINO:
            if lp < KILLED_BY_DOMINO:
                return gmt
            if self.domino and start == gmt and lpivot < k and pivot + p < gmt:
                return perm[pivot + p]
            start, lstart = gmt, low.ldd * a
            stage = KILLED_BY_DISTTREE
        if stage == KILLED_BY_DISTTREE:
            if lp < KILLED_BY_DISTTREE:
                return gmt
            if self._high is not None:
                tmp = self._high.nextpiv(k, pivot, start)
                if tmp != gmt:
                    return perm[tmp]
        return gmt

    def prevpiv(self, k, pivot, start):
        a, p, gmt = self.a, self.p, self.mt
        low = self._low
        ostart, opivot = start, pivot
        start = self._invperm(k, ostart)
        pivot = self._invperm(k, opivot)
        lpivot, rpivot = pivot // p, pivot % p
        lstart = start // p
        perm = self._perm[k]
        ls = self.gettype(k, ostart)
        lp = self.gettype(k, opivot)
        if lp == KILLED_BY_TS:
            return gmt
        stage = ls
        if stage == KILLED_BY_DISTTREE:
            if self._high is not None:
                tmp = self._high.prevpiv(k, pivot, start)
                if tmp != gmt:
                    return perm[tmp]
            start, lstart = pivot, pivot // p
            stage = KILLED_BY_DOMINO
        if stage == KILLED_BY_DOMINO:
            if self.domino and lpivot < k:
                if start == pivot and start + p < gmt:
                    return perm[start + p]
                if lp > KILLED_BY_LOCALTREE:
                    return gmt
            start, lstart = pivot, pivot // p
            stage = KILLED_BY_LOCALTREE
        if stage == KILLED_BY_LOCALTREE:
            if self.domino and lpivot < k:
                return gmt
            tmp = low.prevpiv(k, pivot, lstart // a)
            if tmp * a * p + rpivot >= gmt and tmp == low.ldd - 1:
                tmp = low.prevpiv(k, pivot, tmp)
            if tmp != low.ldd:
                return perm[tmp * a * p + rpivot]
            start = pivot
            stage = KILLED_BY_TS
        if stage == KILLED_BY_TS:
            if start == pivot:
                tmp = lpivot + a - 1 - lpivot % a
                nextp = tmp * p + rpivot
                while pivot < nextp and nextp >= gmt:
                    nextp -= p
            else:
                nextp = start - p
            if pivot < nextp:
                return perm[nextp]
        return gmt


class SystolicTree(QRTree):
    """Systolic 2-level tree (dplasma_systolic_init, src/dplasma_systolic_qr.c): rows >= k+pq are
    TS-killed by k + (m-k) % pq, rows in [k+p, k+pq) TT-killed by k + (m-k) % p, the p rows of the
    band by row k."""

    def __init__(self, mt, nt, p=1, q=1):
        super().__init__(mt, nt, max(1, q), max(1, p), "systolic")

    def getnbgeqrf(self, k):
        return min(self.p * self.a, self.mt - k)

    def getm(self, k, i):
        return k + i

    def gettype(self, k, m):
        p, pq = self.p, self.p * self.a
        if m >= k + pq:
            return KILLED_BY_TS
        return KILLED_BY_LOCALTREE if m >= k + p else KILLED_BY_DISTTREE

    def currpiv(self, k, m):
        p, pq = self.p, self.p * self.a
        t = self.gettype(k, m)
        if t == KILLED_BY_TS:
            return (m - k) % pq + k
        if t == KILLED_BY_LOCALTREE:
            return (m - k) % p + k
        return k

    def nextpiv(self, k, pivot, start):
        p, q, mt = self.p, self.a, self.mt
        pq = p * q
        ls = self.gettype(k, start) if start < mt else -1
        lp = self.gettype(k, pivot)
        stage = ls
        if stage == -1:
            if lp == KILLED_BY_TS:
                return mt
            stage = KILLED_BY_TS
        if stage == KILLED_BY_TS:
            nextp = pivot + pq if start == mt else start + pq
            if nextp < mt:
                return nextp
            start, stage = mt, KILLED_BY_LOCALTREE
        if stage == KILLED_BY_LOCALTREE:
            if lp < KILLED_BY_DISTTREE:
                return mt
            nextp = pivot + p if start == mt else start + p
            if k + p <= nextp < min(k + pq, mt):
                return nextp
            start, stage = mt, KILLED_BY_DISTTREE
        if stage == KILLED_BY_DISTTREE:
            if pivot > k:
                return mt
            nextp = pivot + 1 if start == mt else start + 1
            if nextp < k + p:
                return nextp
        return mt

    def prevpiv(self, k, pivot, start):
        p, q, mt = self.p, self.a, self.mt
        pq = p * q
        rpivot = pivot % pq
        ls, lp = self.gettype(k, start), self.gettype(k, pivot)
        if lp == KILLED_BY_TS:
            return mt
        stage = ls
        if stage == KILLED_BY_DISTTREE:
            if pivot == k:
                if start == pivot:
                    nextp = start + p - 1
                    while pivot < nextp and nextp >= mt:
                        nextp -= 1
                else:
                    nextp = start - 1
                if pivot < nextp < k + p:
                    return nextp
            start, stage = pivot, KILLED_BY_LOCALTREE
        if stage == KILLED_BY_LOCALTREE:
            if lp > KILLED_BY_LOCALTREE:
                if start == pivot:
                    nextp = start + (q - 1) * p
                    while pivot < nextp and nextp >= mt:
                        nextp -= p
                else:
                    nextp = start - p
                if pivot < nextp < k + pq:
                    return nextp
            start, stage = pivot, KILLED_BY_TS
        if stage == KILLED_BY_TS:
            if lp > KILLED_BY_TS:
                if start == pivot:
                    nextp = mt - (mt - rpivot - 1) % pq - 1
                    while pivot < nextp and nextp >= mt:
                        nextp -= pq
                else:
                    nextp = start - pq
                if pivot < nextp:
                    return nextp
        return mt


class SVDTree(QRTree):
    """Adaptive tree of the bidiagonal reduction (dplasma_svd_init, src/dplasma_hqr.c:1975-2700): per
    panel k the TS domain size a_k is chosen so that every core keeps at least ``ratio`` columns of TS
    work (a_k ~ ceil(mt-k, p) (nt-k) / (ratio cores), balanced), each process row's domain heads are
    reduced by a per-panel greedy, and the p-row band by ``hlvl`` (default fibonacci)."""

    def __init__(self, mt, nt, hlvl=GREEDY_TREE, p=1, nbcores_per_node=1, ratio=1, nodes=None):
        p = max(p, 1)
        super().__init__(mt, nt, -1, p, "svd")
        self.hlvl = hlvl
        nodes = p if nodes is None else nodes
        cores = max(1, nbcores_per_node) * max(1, nodes // p)
        ratio = max(1, ratio)
        min_mn = min(mt, nt)
        self._sa, self._sldd = [], []      # per panel: domain size, number of domains
        for k in range(min_mn):
            height = -(-(mt - k) // p)
            a = max(height * (nt - k) // (ratio * cores), 1)
            j = -(-height // a)
            a = -(-(mt - k) // j)
            self._sa.append(a)
            self._sldd.append(-(-mt // (p * a)))
        self._lowtab = []                  # [rank][k] -> greedy pivot column
        for r in range(p):
            cols = []
            for k in range(min_mn):
                a, ldd = self._sa[k], self._sldd[k]
                col = [0] * max(ldd, 1)
                nT = max(ldd - (k + p - 1 - r) // (p * a), 0)
                nZ = 0
                while nZ < nT - 1:
                    h = (nT - nZ) // 2
                    top = ldd - nZ - 1
                    nZ += h
                    for jj in range(top, top - h, -1):
                        col[jj] = jj - h
                cols.append(col)
            self._lowtab.append(cols)
        self._high = _high_tree(hlvl, mt, -1, p, False, min_mn, default_flat=False) if p > 1 else None

    def _ka(self, k, row):
        a = self._sa[k]
        return (k + self.p - 1 - row % self.p) // self.p // a

    def getnbgeqrf(self, k):
        p, gmt, a = self.p, self.mt, self._sa[k]
        pa = p * a
        nb2 = _nbextra1(k, pa, p)
        nb11 = (k + p + pa - 1) // pa * pa
        nb12 = (gmt // pa) * pa
        d = nb12 - nb11
        nb1 = (d // a if d >= 0 else -((-d) // a)) + min(p, gmt - nb12)
        return min(nb1 + nb2 + p, gmt - k)

    def getm(self, k, i):
        p, a = self.p, self._sa[k]
        pa = p * a
        nb23 = p + _nbextra1(k, pa, p)
        if i < nb23:
            return k + i
        j = i - nb23
        pos1 = (p + k + pa - 1) // pa * pa
        return pos1 + (j // p) * pa + j % p

    def gettype(self, k, m):
        p, a = self.p, self._sa[k]
        if m < k + p:
            return KILLED_BY_DISTTREE
        return KILLED_BY_LOCALTREE if (m // p) % a == 0 else KILLED_BY_TS

    def _low_currpiv(self, k, m):
        return self._lowtab[m % self.p][k][(m // self.p) // self._sa[k]]

    def _low_nextpiv(self, k, piv, s):
        col, a, ldd = self._lowtab[piv % self.p][k], self._sa[k], self._sldd[k]
        ppa, ka = piv // (self.p * a), self._ka(k, piv)
        for i in range(s - 1, ka, -1):
            if col[i] == ppa:
                return i
        return ldd

    def _low_prevpiv(self, k, piv, s):
        col, a, ldd = self._lowtab[piv % self.p][k], self._sa[k], self._sldd[k]
        ppa = piv // self.p // a
        for i in range(s + 1, ldd):
            if col[i] == ppa:
                return i
        return ldd

    def currpiv(self, k, m):
        p, gmt, a = self.p, self.mt, self._sa[k]
        lm, rank = m // p, m % p
        t = self.gettype(k, m)
        tmpk = k // (p * a)
        if t == KILLED_BY_TS:
            tmp = lm // a
            return k + (m - k) % p if tmp == tmpk else tmp * a * p + rank
        if t == KILLED_BY_LOCALTREE:
            tmp = self._low_currpiv(k, m)
            return k + (m - k) % p if tmp == tmpk else tmp * a * p + rank
        return self._high.currpiv(k, m) if self._high is not None else gmt

    def nextpiv(self, k, pivot, start):
        p, gmt = self.p, self.mt
        a, ldd = self._sa[k], self._sldd[k]
        rpivot = pivot % p
        lstart = ldd * a if start == gmt else start // p
        ls = self.gettype(k, start) if start < gmt else -1
        lp = self.gettype(k, pivot)
        stage = ls
        if stage == -1:
            if lp == KILLED_BY_TS:
                return gmt
            stage = KILLED_BY_TS
        if stage == KILLED_BY_TS:
            nextp = pivot + p if start == gmt else start + p
            if nextp < gmt and nextp < pivot + a * p and (nextp // p) % a != 0:
                return nextp
            start, lstart, stage = gmt, ldd * a, KILLED_BY_LOCALTREE
        if stage == KILLED_BY_LOCALTREE:
            tmp = self._low_nextpiv(k, pivot, lstart // a)
            if tmp * a * p + rpivot >= gmt and tmp == ldd - 1:
                tmp = self._low_nextpiv(k, pivot, tmp)
            if tmp != ldd:
                return tmp * a * p + rpivot
            start, lstart, stage = gmt, ldd * a, KILLED_BY_DISTTREE
        if stage == KILLED_BY_DISTTREE:
            if lp < KILLED_BY_DISTTREE:
                return gmt
            if self._high is not None:
                tmp = self._high.nextpiv(k, pivot, start)
                if tmp != gmt:
                    return tmp
        return gmt

    def prevpiv(self, k, pivot, start):
        p, gmt = self.p, self.mt
        a, ldd = self._sa[k], self._sldd[k]
        lpivot, rpivot, lstart = pivot // p, pivot % p, start // p
        ls, lp = self.gettype(k, start), self.gettype(k, pivot)
        if lp == KILLED_BY_TS:
            return gmt
        stage = ls
        if stage == KILLED_BY_DISTTREE:
            if self._high is not None:
                tmp = self._high.prevpiv(k, pivot, start)
                if tmp != gmt:
                    return tmp
            start, lstart, stage = pivot, pivot // p, KILLED_BY_LOCALTREE
        if stage == KILLED_BY_LOCALTREE:
            tmp = self._low_prevpiv(k, pivot, lstart // a)
            if tmp * a * p + rpivot >= gmt and tmp == ldd - 1:
                tmp = self._low_prevpiv(k, pivot, tmp)
            if tmp != ldd:
                return tmp * a * p + rpivot
            start, stage = pivot, KILLED_BY_TS
        if stage == KILLED_BY_TS:
            if start == pivot:
                tmp = lpivot + a - 1 - lpivot % a
                nextp = tmp * p + rpivot
                while pivot < nextp and nextp >= gmt:
                    nextp -= p
            else:
                nextp = start - p
            if pivot < nextp:
                return nextp
        return gmt


class FlatTree(HQRTree):
    """PLASMA flat TS tree (plain geqrf): one domain covering the whole panel."""

    def __init__(self, mt, nt):
        super().__init__(mt, nt, llvl=FLAT_TREE, hlvl=FLAT_TREE, a=mt, p=1)
        self.name = "flat"


# ----------------------------------------------------------------------------- reference-style constructors
def _dims(trans, A):
    return (A.mt, A.nt) if trans == dplasmaNoTrans else (A.nt, A.mt)


def hqr_init(trans, A, llvl=GREEDY_TREE, hlvl=FLAT_TREE, a=1, p=None, domino=False, tsrr=False) -> HQRTree:
    """``dplasma_hqr_init(qrtree, trans, A, type_llvl, type_hlvl, a, p, domino, tsrr)``.

    trans = NoTrans builds a QR tree over A's tile rows; ConjTrans an LQ tree
    over its tile columns.  p defaults to the process-grid rows (QR) / columns (LQ)."""
    mt, nt = _dims(trans, A)
    if p is None or p <= 0:
        p = A.grid.P if trans == dplasmaNoTrans else A.grid.Q
    return HQRTree(mt, nt, llvl, hlvl, -1 if a == -1 else max(a or 1, 1), p, domino, tsrr)


def systolic_init(trans, A, p=1, q=1) -> SystolicTree:
    mt, nt = _dims(trans, A)
    return SystolicTree(mt, nt, p, q)


def svd_init(trans, A, hlvl=GREEDY_TREE, p=1, nbcores_per_node=1, ratio=1) -> SVDTree:
    """``dplasma_svd_init(qrtree, trans, A, type_hlvl, p, nbthread_per_node, ratio)``: the core count
    of the adaptive domain size is nbthread_per_node * (nodes / p), nodes = the descriptor's ranks."""
    mt, nt = _dims(trans, A)
    g = getattr(A, "grid", None)
    nodes = g.P * g.Q if g is not None else max(p, 1)
    return SVDTree(mt, nt, hlvl, p, nbcores_per_node, ratio, nodes=nodes)


def qrtree_check(A, qrtree: QRTree) -> int:
    return qrtree.check()
