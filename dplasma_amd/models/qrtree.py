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


class HQRTree(QRTree):
    """Hierarchical tree (dplasma_hqr_init, src/dplasma_hqr.c:1670-1948).

    Rows of panel k are grouped by "process row" ``m % p``; inside a process
    row, consecutive local rows form TS domains of ``a`` tiles (flat TS tree,
    no communication); the domain heads are reduced by the low-level tree
    ``llvl`` (local TT kernels); the process-row survivors are reduced by the
    high-level tree ``hlvl`` (distributed TT kernels, one tile-row exchange per
    elimination).  ``domino``: the high level is a flat TT chain (type 2),
    which pipelines consecutive panels; ``tsrr``: TS domains are formed
    round-robin over the local rows instead of contiguously."""

    def __init__(self, mt, nt, llvl=GREEDY_TREE, hlvl=FLAT_TREE, a=1, p=1, domino=False, tsrr=False):
        self.llvl, self.hlvl, self.domino, self.tsrr = llvl, hlvl, bool(domino), bool(tsrr)
        a = max(1, min(a, mt)) if a > 0 else 1
        p = max(1, p)
        super().__init__(mt, nt, a, p, "hqr")

    def _plan(self, k):
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
