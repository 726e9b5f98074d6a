"""Reduction trees for hierarchical tile QR/LQ (pure integer logic).

Reference: ``src/include/dplasma/qr_param.h:18-148`` (the ``dplasma_qrtree_t``
query interface), ``src/dplasma_hqr.c`` (3-level HQR trees), ``src/dplasma_systolic_qr.c``
(systolic 2-level tree) and ``src/dplasma_hqr_dbg.c`` (validation / printers).

Design: instead of closed-form index functions evaluated inside a JDF, a tree
here is an explicit *elimination plan* per panel k:

* ``heads(k)``  -- the rows that get a GEQRT at step k (never TS-killed),
* ``kills(k)``  -- ordered list of ``(piv, m, type)``: row m is annihilated by
  row piv with a TS kernel (type 0) or a TT kernel (types 1 local tree,
  2 domino, 3 distributed tree), in a valid program order (a row finishes all
  of its own kills before it is killed).

The tile-DAG runtime (``runtime/dag.py``) turns the plan into a leveled DAG, so
tree parallelism (all eliminations of one tree round) automatically lands in
the same batched launch.  The reference's query functions (getnbgeqrf, getm,
geti, gettype, currpiv, nextpiv, prevpiv) are provided on top of the plans.

Tree shapes over an ordered row list (element 0 is the survivor):
  FLAT       sequential: r0 kills r1, r2, ...
  GREEDY     each round the bottom half is killed by the top half (log depth)
  FIBONACCI  each round kills a Fibonacci-limited number of bottom rows
  BINARY     pairwise at doubling distance (r0<-r1, r2<-r3; r0<-r2; ...)
  GREEDY1P   greedy that keeps one annihilator per round and process row group
"""
from __future__ import annotations

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
    """Explicit elimination plans for every panel (see module docstring).

    ``mt``/``nt``: tile rows/cols of the (logical) matrix being factored
    (for an LQ tree built with trans=ConjTrans these are A.nt / A.mt)."""

    def __init__(self, mt: int, nt: int, a: int, p: int, name: str):
        self.mt, self.nt, self.a, self.p = mt, nt, a, p
        self.name = name
        self._heads: Dict[int, List[int]] = {}
        self._kills: Dict[int, List[Tuple[int, int, int]]] = {}
        self._plan_all()
        self._index()

    # subclasses fill one panel
    def _plan(self, k: int):
        raise NotImplementedError

    def _plan_all(self):
        for k in range(min(self.mt, self.nt)):
            heads, kills = self._plan(k)
            self._heads[k] = sorted(heads)
            self._kills[k] = kills

    def _index(self):
        self._type, self._piv, self._seq = {}, {}, {}
        for k, kl in self._kills.items():
            for (p, m, t) in kl:
                self._type[(k, m)] = t
                self._piv[(k, m)] = p
                self._seq.setdefault((k, p), []).append(m)

    # ------------------------------------------------------------ plan access
    def heads(self, k: int) -> List[int]:
        return self._heads[k]

    def kills(self, k: int) -> List[Tuple[int, int, int]]:
        return self._kills[k]

    # ------------------------------------------------------------ reference query interface
    def getnbgeqrf(self, k: int) -> int:
        return len(self._heads[k])

    def getm(self, k: int, i: int) -> int:
        return self._heads[k][i]

    def geti(self, k: int, m: int) -> int:
        return self._heads[k].index(m)

    def gettype(self, k: int, m: int) -> int:
        """Kill type of row m at step k (0 TS, >0 TT); -1 for the panel's diagonal row."""
        return self._type.get((k, m), -1)

    def currpiv(self, k: int, m: int) -> int:
        return self._piv.get((k, m), self.mt)

    def nextpiv(self, k: int, p: int, m: int) -> int:
        """Next row killed by p after m at step k (m = mt: first one); mt if none."""
        seq = self._seq.get((k, p), [])
        if m == self.mt:
            return seq[0] if seq else self.mt
        i = seq.index(m)
        return seq[i + 1] if i + 1 < len(seq) else self.mt

    def prevpiv(self, k: int, p: int, m: int) -> int:
        """Previous row killed by p before m at step k (m = p: the last one); mt if none."""
        seq = self._seq.get((k, p), [])
        if m == p:
            return seq[-1] if seq else self.mt
        i = seq.index(m)
        return seq[i - 1] if i > 0 else self.mt

    # ------------------------------------------------------------ validation / debug
    def check(self) -> int:
        """Validate the plans (dplasma_qrtree_check analogue): 0 if valid, else raises."""
        for k in range(min(self.mt, self.nt)):
            heads = set(self._heads[k])
            if k not in heads:
                raise AssertionError(f"panel {k}: diagonal row is not a GEQRT head")
            killed = set()
            alive = set(range(k, self.mt))
            for (p, m, t) in self._kills[k]:
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
                killed.add(m)
            if alive - killed != {k}:
                raise AssertionError(f"panel {k}: survivors {sorted(alive - killed)} != [{k}]")
            for m in range(k + 1, self.mt):
                if m not in heads and self._type.get((k, m)) != KILLED_BY_TS:
                    raise AssertionError(f"panel {k}: row {m} neither GEQRT'ed nor TS-killed")
        return 0

    def depth(self, k: int) -> int:
        """Critical path (rounds) of panel k's elimination (TS kills count 1 each along a chain)."""
        t = {m: 0 for m in range(k, self.mt)}
        for (p, m, _) in self._kills[k]:
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
            for (p, m, t) in self._kills[kk]:
                style = "solid" if t else "dashed"
                out.append(f'  "k{kk}_{m}" -> "k{kk}_{p}" [style={style},label="{t}"];')
        out.append("}")
        return "\n".join(out)

    def __repr__(self):
        return f"QRTree({self.name}, mt={self.mt}, nt={self.nt}, a={self.a}, p={self.p})"


def _lowbit_piv(d: int) -> int:
    """Binary tree over offsets: offset d > 0 is killed by d minus its lowest set bit."""
    return d - (d & -d)


def _fib_piv(d: int) -> int:
    """Fibonacci (order 1) tree over offsets: groups of 1, 2, 3, ... consecutive offsets, each
    offset killed by the one ``group size`` above it (dplasma_hqr.c fibonacci ipiv, first column)."""
    f, start = 1, 1
    while d >= start + f:
        start += f
        f += 1
    return d - f


def _greedy_low_table(ldd: int, min_mn: int, p: int, a: int):
    """Pivot domain index of domain j at panel k for process row r, tab[r][k][j], of the reference's
    coarse-grained greedy low-level tree (dplasma_hqr.c hqr_low_greedy_init, non-domino): per panel
    column, half of the domains still to be annihilated are killed by the ones just above them,
    columns advancing as soon as their predecessor has produced enough triangles.  Re-implemented
    here because identical elimination trees are the point (the tree defines the V/T layout)."""
    pa = p * a
    tab = [[[0] * ldd for _ in range(min_mn)] for _ in range(p)]
    for r in range(p):
        todo = []
        for k in range(min_mn):
            v = max(ldd - (k + p - 1 - r) // pa, 0)
            if v == 0:
                break
            todo.append(v)
        lmin = len(todo)
        if lmin == 0:
            continue
        nt_ = [0] * lmin
        nz = [0] * lmin
        nt_[0] = ldd
        k = first = 0
        guard = 0
        while not (nt_[lmin - 1] == todo[lmin - 1] and nz[lmin - 1] + 1 == nt_[lmin - 1]) and first < lmin:
            guard += 1
            if guard > 10 * (ldd + 2) * (lmin + 2):
                raise RuntimeError("greedy tree schedule did not converge")
            h = (nt_[k] - nz[k]) // 2
            if h == 0:
                while first < lmin and nt_[first] == todo[first] and nz[first] + 1 == nt_[first]:
                    if first < lmin - 1 and first % pa != (a - 1) * p + r:
                        nt_[first + 1] += 1
                    first += 1
                k = first
                continue
            if k < lmin - 1:
                nt_[k + 1] += h
            top = ldd - nz[k] - 1
            for j in range(top, top - h, -1):
                tab[r][k][j] = j - h
            nz[k] += h
            k += 1
            if k > lmin - 1:
                k = first
    return tab


def _greedy_high_table(mt: int, min_mn: int, p: int):
    """tab[k][d]: pivot row of band row k+d at panel k of the reference's greedy high-level tree
    (dplasma_hqr.c hqr_high_greedy_init)."""
    tab = [[0] * p for _ in range(min_mn)]
    nt_ = [0] * min_mn
    nz = [0] * min_mn
    nt_[0] = mt
    nz[0] = max(mt - p, 0)
    for k in range(1, min_mn):
        nt_[k] = nz[k] = max(mt - k - p, 0)
    k = first = 0
    guard = 0
    while not (nt_[min_mn - 1] == mt - (min_mn - 1) and nz[min_mn - 1] + 1 == nt_[min_mn - 1]) and first < min_mn:
        guard += 1
        if guard > 10 * (mt + 2) * (min_mn + 2):
            raise RuntimeError("greedy tree schedule did not converge")
        h = (nt_[k] - nz[k]) // 2
        if h == 0:
            while first < min_mn and nt_[first] == mt - first and nz[first] + 1 == nt_[first]:
                first += 1
            k = first
            continue
        top = mt - nz[k] - 1
        nz[k] += h
        if k < min_mn - 1:
            nt_[k + 1] = nz[k]
        for j in range(top, top - h, -1):
            tab[k][j - k] = j - h
        k += 1
        if k > min_mn - 1:
            k = first
    return tab


class HQRTree(QRTree):
    """Hierarchical tree (dplasma_hqr_init, src/dplasma_hqr.c:1670-1948).

    Rows of panel k are grouped by "process row" ``m % p``.  Reference semantics (gettype /
    currpiv, dplasma_hqr.c:299-322, 1241-1311), reproduced exactly for the non-domino, non-tsrr trees:
    the p rows [k, k+p) are the distributed (type 3) rows, reduced by the high-level tree ``hlvl``;
    below them, TS domains are the GLOBALLY aligned groups of ``a`` consecutive local rows
    ((m / p) / a is the domain index), each killed by its first row (type 1) -- except the domain
    containing the diagonal macro-tile, whose rows the type-3 row of their process row kills; the
    domain heads of a process row are reduced by the low-level tree ``llvl`` over domain indices
    (flat, binary, fibonacci and greedy as the reference defines them; greedy1p uses the per-panel
    greedy shape).  ``domino``: the high level is a flat TT chain (type 2) pipelining consecutive
    panels; ``tsrr``: TS domains formed round-robin over the local rows (both per-panel shapes)."""

    def __init__(self, mt, nt, llvl=GREEDY_TREE, hlvl=FLAT_TREE, a=1, p=1, domino=False, tsrr=False):
        self.llvl, self.hlvl, self.domino, self.tsrr = llvl, hlvl, bool(domino), bool(tsrr)
        a = max(1, min(a, mt)) if a > 0 else 1
        p = max(1, p)
        self._min_mn = min(mt, nt)
        self._ldd = -(-mt // (p * a))
        self._glow = _greedy_low_table(self._ldd, self._min_mn, p, a) if llvl == GREEDY_TREE else None
        self._ghigh = _greedy_high_table(mt, self._min_mn, p) if hlvl == GREEDY_TREE and p > 1 else None
        super().__init__(mt, nt, a, p, "hqr")

    def _plan(self, k):
        if self.domino or self.tsrr:
            return self._plan_local(k)
        return self._plan_aligned(k)

    def _low_piv(self, k, r, j, k_a):
        """Pivot domain index of domain j (> k_a) of process row r at panel k."""
        t = self.llvl
        if t == FLAT_TREE:
            return k_a
        if t == BINARY_TREE:
            return k_a + _lowbit_piv(j - k_a)
        if t == FIBONACCI_TREE:
            return k_a + _fib_piv(j - k_a)
        if t == GREEDY_TREE:
            return self._glow[r][k][j]
        return None   # greedy1p: per-panel shape

    def _high_piv(self, k, m):
        t, d = self.hlvl, m - k
        if t == FLAT_TREE:
            return k
        if t == BINARY_TREE:
            return k + _lowbit_piv(d)
        if t == FIBONACCI_TREE:
            return k + _fib_piv(d)
        if t == GREEDY_TREE:
            return self._ghigh[k][d]
        return None

    def _plan_aligned(self, k):
        a, p, mt = self.a, self.p, self.mt
        pa = p * a
        tmpk = k // pa
        band = [m for m in range(k, min(mt, k + p))]          # type 3 rows, one per process row
        t_of = {m % p: m for m in band}
        heads, ts, low, high = list(band), [], [], []
        by_res = {r: [] for r in t_of}                        # aligned heads (type 1) per process row
        for m in range(k + p, mt):
            r, li = m % p, m // p
            if li % a == 0:
                heads.append(m)
                by_res[r].append(m)
            else:
                idx = li // a
                ts.append((t_of[r] if idx == tmpk else idx * pa + r, m, KILLED_BY_TS))
        for r, hs in by_res.items():
            if not hs:
                continue
            k_a = (k + p - 1 - r) // p // a
            doms = [t_of[r]] + hs
            idx_of = {m: (k_a if m == t_of[r] else m // pa) for m in doms}
            row_of = {idx_of[m]: m for m in doms}
            pairs = []
            for m in sorted(hs, reverse=True):
                j = idx_of[m]
                pj = self._low_piv(k, r, j, k_a)
                if pj is None:
                    pairs = None
                    break
                pairs.append((row_of.get(pj, t_of[r]), m))
            if pairs is None:
                pairs = tree_pairs(doms, self.llvl)
            low += [(pv, m, KILLED_BY_LOCALTREE) for (pv, m) in pairs]
        hp = []
        for m in sorted(band[1:], reverse=True):
            pv = self._high_piv(k, m)
            if pv is None:
                hp = None
                break
            hp.append((pv, m))
        if hp is None:
            hp = tree_pairs(band, self.hlvl)
        high = [(pv, m, KILLED_BY_DISTTREE) for (pv, m) in hp]
        return heads, ts + low + high

    def _plan_local(self, k):
        a, p = self.a, self.p
        heads, kills = [], []
        roots = []
        for q in range(p):
            pr = (k + q) % p  # process rows in order starting with the diagonal's
            local = [m for m in range(k, self.mt) if m % p == pr]
            if not local:
                continue
            nd = (len(local) + a - 1) // a
            if self.tsrr:
                doms = [local[i::nd] for i in range(nd)]
            else:
                doms = [local[i * a:(i + 1) * a] for i in range(nd)]
            dheads = []
            for d in doms:
                dheads.append(d[0])
                kills += [(d[0], m, KILLED_BY_TS) for m in d[1:]]
            heads += dheads
            kills += [(pv, m, KILLED_BY_LOCALTREE) for (pv, m) in tree_pairs(sorted(dheads), self.llvl)]
            roots.append(min(dheads))
        if self.domino:
            kills += [(pv, m, KILLED_BY_DOMINO) for (pv, m) in tree_pairs(roots, FLAT_TREE)]
        else:
            kills += [(pv, m, KILLED_BY_DISTTREE) for (pv, m) in tree_pairs(roots, self.hlvl)]
        return heads, kills


class SystolicTree(QRTree):
    """Systolic 2-level tree (dplasma_systolic_init, src/dplasma_systolic_qr.c:56-120):
    rows >= k+p*q are TS-killed by row k + (m-k) % (p*q); rows in [k+p, k+p*q) are
    TT-killed by k + (m-k) % p; rows in (k, k+p) by row k (flat, type 3)."""

    def __init__(self, mt, nt, p=1, q=1):
        super().__init__(mt, nt, max(1, q), max(1, p), "systolic")

    def _plan(self, k):
        p, q = self.p, self.a
        pq = p * q
        heads = list(range(k, min(self.mt, k + pq)))
        kills = []
        for m in range(k + pq, self.mt):
            kills.append(((m - k) % pq + k, m, KILLED_BY_TS))
        for m in range(k + p, min(self.mt, k + pq)):
            kills.append(((m - k) % p + k, m, KILLED_BY_LOCALTREE))
        for m in range(k + 1, min(self.mt, k + p)):
            kills.append((k, m, KILLED_BY_DISTTREE))
        return heads, kills


class SVDTree(HQRTree):
    """Adaptive tree for the bidiagonal reduction (dplasma_svd_init, src/dplasma_hqr.c:1975-2700):
    per panel, the TS domain size shrinks with the remaining rows so that every
    process row keeps about ``ratio * nbcores_per_node`` independent domains."""

    def __init__(self, mt, nt, hlvl=GREEDY_TREE, p=1, nbcores_per_node=1, ratio=1):
        self.cores, self.ratio = max(1, nbcores_per_node), max(1, ratio)
        super().__init__(mt, nt, llvl=GREEDY_TREE, hlvl=hlvl, a=1, p=p)

    def _plan(self, k):
        rows_per_proc = max(1, (self.mt - k + self.p - 1) // self.p)
        self.a = max(1, rows_per_proc // (self.cores * self.ratio))
        return super()._plan(k)


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
    return HQRTree(mt, nt, llvl, hlvl, a if a and a > 0 else 1, p, domino, tsrr)


def systolic_init(trans, A, p=1, q=1) -> SystolicTree:
    mt, nt = _dims(trans, A)
    return SystolicTree(mt, nt, p, q)


def svd_init(trans, A, hlvl=GREEDY_TREE, p=1, nbcores_per_node=1, ratio=1) -> SVDTree:
    mt, nt = _dims(trans, A)
    return SVDTree(mt, nt, hlvl, p, nbcores_per_node, ratio)


def qrtree_check(A, qrtree: QRTree) -> int:
    return qrtree.check()
