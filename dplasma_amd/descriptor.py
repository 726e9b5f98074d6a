"""Tiled matrix descriptors: 2-D block-cyclic distribution over a P x Q grid.

Equivalent of the reference's data layer (parsec_matrix_block_cyclic_init /
_lapack_init / sym_block_cyclic used throughout ``tests/testing_z*.c``, e.g.
``tests/testing_zpotrf.c:42-45``, and the shape/location logic of
``src/utils/dplasma_lapack_adtt.c``), re-designed for one process per GPU:

* Every rank owns the tiles (m, n) with ``prow(m) == my_prow`` and
  ``pcol(n) == my_pcol`` where ``prow(m) = (m // kp + ip) % P`` and
  ``pcol(n) = (n // kq + jq) % Q`` (k-cyclic repetition kp/kq, grid offsets
  ip/jq).  Rank = prow * Q + pcol (row-major grid).
* Local tiles live in ONE contiguous torch tensor on the rank's device (GPU
  HBM, or host memory for the CPU path):
    - TILE storage: each mb x nb tile contiguous (column-major, ld = mb); local
      tiles ordered column-major over the local tile grid, so the local part of
      a tile column is one contiguous slab -- panels are sent without packing;
    - LAPACK storage: the local matrix is column-major with leading dimension
      ``lld`` (ScaLAPACK layout); tile (i, j) starts at i*mb + j*nb*lld.
* Tile addressing is (element offset, leading dimension), which is exactly
  what the batched GPU kernels consume (csrc/kernels/common.h item records).
* Sub-matrix views (tile-aligned ``i, j`` offsets) share storage.

Edge tiles are ragged (``tile_rows/cols``), like the reference's
``CLEAN_MB/NB`` (src/floputils.h).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import torch

from .constants import STORAGE_LAPACK, STORAGE_TILE, DTYPE_PREC, dplasmaLower, dplasmaUpper, dplasmaUpperLower


def _cdiv(a, b):
    return (a + b - 1) // b


@dataclass
class Grid:
    """P x Q process grid with k-cyclic repetition and offsets."""
    P: int = 1
    Q: int = 1
    kp: int = 1
    kq: int = 1
    ip: int = 0
    jq: int = 0

    def prow(self, m: int) -> int:
        return (m // self.kp + self.ip) % self.P

    def pcol(self, n: int) -> int:
        return (n // self.kq + self.jq) % self.Q

    def rank(self, pr: int, pc: int) -> int:
        return pr * self.Q + pc

    def coords(self, rank: int):
        return rank // self.Q, rank % self.Q


class TiledMatrix:
    """A distributed tiled matrix (one rank's view).

    Parameters mirror ``parsec_matrix_block_cyclic_init(dc, type, storage,
    rank, mb, nb, lm, ln, i, j, m, n, P, Q, kp, kq, ip, jq)``.
    """

    def __init__(self, dtype: torch.dtype, mb: int, nb: int, lm: int, ln: int, *, P: int = 1, Q: int = 1,
                 kp: int = 1, kq: int = 1, ip: int = 0, jq: int = 0, rank: int = 0, device="cpu",
                 storage: str = STORAGE_TILE, lld: Optional[int] = None, uplo: int = dplasmaUpperLower,
                 data: Optional[torch.Tensor] = None, alloc: bool = True, name: str = "A"):
        if mb <= 0 or nb <= 0:
            raise ValueError("tile sizes must be positive")
        self.dtype = dtype
        self.prec = DTYPE_PREC.get(dtype, 'i')  # integer descriptors (IPIV) use 'i'
        self.mb, self.nb = mb, nb
        self.lm, self.ln = lm, ln          # full matrix extent
        self.lmt, self.lnt = _cdiv(lm, mb), _cdiv(ln, nb)
        self.grid = Grid(P, Q, kp, kq, ip, jq)
        self.rank = rank
        self.myrow, self.mycol = self.grid.coords(rank) if rank < P * Q else (-1, -1)
        self.device = torch.device(device)
        self.storage = storage
        self.uplo = uplo                    # which triangle is meaningful (sym_block_cyclic)
        self.name = name
        # view parameters (full matrix by default)
        self.i, self.j, self.m, self.n = 0, 0, lm, ln
        self.it0, self.jt0 = 0, 0
        # local tile grid: global tile rows/cols owned by this rank, in order
        self.rows = [t for t in range(self.lmt) if self.grid.prow(t) == self.myrow]
        self.cols = [t for t in range(self.lnt) if self.grid.pcol(t) == self.mycol]
        self.lrow = {t: k for k, t in enumerate(self.rows)}
        self.lcol = {t: k for k, t in enumerate(self.cols)}
        self.llmt, self.llnt = len(self.rows), len(self.cols)
        # local element extents (LAPACK storage)
        self.llm = sum(self._grows(t) for t in self.rows)
        self.lln = sum(self._gcols(t) for t in self.cols)
        if storage == STORAGE_TILE:
            self.ld = mb
            self.nelem = self.llmt * self.llnt * mb * nb
        elif storage == STORAGE_LAPACK:
            self.ld = max(1, lld if lld is not None else self.llm)
            if self.ld < self.llm:
                raise ValueError("lld < local rows")
            self.nelem = self.ld * max(self.lln, 0)
        else:
            raise ValueError(storage)
        if data is not None:
            if data.numel() < self.nelem:
                raise ValueError("user buffer too small for the descriptor")
            self.data = data
        elif alloc:
            self.data = torch.zeros(max(self.nelem, 1), dtype=dtype, device=self.device)
        else:
            self.data = None
        self._parent = None

    # ------------------------------------------------------------ geometry
    def _grows(self, gt: int) -> int:
        return min(self.mb, self.lm - gt * self.mb)

    def _gcols(self, gt: int) -> int:
        return min(self.nb, self.ln - gt * self.nb)

    @property
    def mt(self) -> int:
        return _cdiv(self.m, self.mb) if self.m > 0 else 0

    @property
    def nt(self) -> int:
        return _cdiv(self.n, self.nb) if self.n > 0 else 0

    @property
    def P(self):
        return self.grid.P

    @property
    def Q(self):
        return self.grid.Q

    def tile_rows(self, m: int) -> int:
        """Rows of view tile m (ragged last tile)."""
        return min(self.mb, self.m - m * self.mb)

    def tile_cols(self, n: int) -> int:
        return min(self.nb, self.n - n * self.nb)

    def rank_of(self, m: int, n: int) -> int:
        gm, gn = m + self.it0, n + self.jt0
        return self.grid.rank(self.grid.prow(gm), self.grid.pcol(gn))

    def is_local(self, m: int, n: int) -> bool:
        return self.rank_of(m, n) == self.rank

    def row_is_local(self, m: int) -> bool:
        return self.grid.prow(m + self.it0) == self.myrow

    def col_is_local(self, n: int) -> bool:
        return self.grid.pcol(n + self.jt0) == self.mycol

    def offset(self, m: int, n: int) -> int:
        """Element offset of local view tile (m, n) in ``self.data``."""
        gm, gn = m + self.it0, n + self.jt0
        il, jl = self.lrow[gm], self.lcol[gn]
        if self.storage == STORAGE_TILE:
            return (jl * self.llmt + il) * self.mb * self.nb
        return il * self.mb + jl * self.nb * self.ld

    def tile(self, m: int, n: int) -> torch.Tensor:
        """Column-major view (rows x cols) of local tile (m, n)."""
        r, c = self.tile_rows(m), self.tile_cols(n)
        return torch.as_strided(self.data, (r, c), (1, self.ld), self.offset(m, n))

    def local_tiles(self, uplo: int = dplasmaUpperLower):
        """Iterate (m, n) over local view tiles, optionally restricted to a triangle (tile-wise)."""
        for n in range(self.nt):
            if not self.col_is_local(n):
                continue
            for m in range(self.mt):
                if not self.row_is_local(m):
                    continue
                if uplo == dplasmaLower and m < n:
                    continue
                if uplo == dplasmaUpper and m > n:
                    continue
                yield m, n

    # ------------------------------------------------------------ views
    def submatrix(self, i: int, j: int, m: int, n: int) -> "TiledMatrix":
        """View of rows i:i+m, cols j:j+n (i, j multiples of mb, nb), sharing storage."""
        if i % self.mb or j % self.nb:
            raise ValueError("submatrix offsets must be tile aligned")
        if self.i + i + m > self.lm or self.j + j + n > self.ln:
            raise ValueError("submatrix out of range")
        v = object.__new__(TiledMatrix)
        v.__dict__.update(self.__dict__)
        v.i, v.j, v.m, v.n = self.i + i, self.j + j, m, n
        v.it0, v.jt0 = v.i // self.mb, v.j // self.nb
        v._parent = self
        return v

    def tile_desc(self, m: int, n: int, hnb: int) -> "TiledMatrix":
        """One-process descriptor over local tile (m, n) itself, tiled hnb x hnb (LAPACK storage,
        ld = this descriptor's ld, sharing storage): the operand of a recursive sub-taskpool
        (reference: the small_descA of parsec_recursivecall, src/zpotrf_L.jdf:148-172)."""
        r, c = self.tile_rows(m), self.tile_cols(n)
        off = self.offset(m, n)
        return TiledMatrix(self.dtype, hnb, hnb, r, c, device=self.device, storage=STORAGE_LAPACK, lld=self.ld,
                           uplo=self.uplo, data=self.data[off:], name=f"{self.name}({m},{n})")

    def like(self, dtype=None, storage=None, alloc=True, name=None, lm=None, ln=None) -> "TiledMatrix":
        """Same distribution/tiling, new storage (full matrix, not a view)."""
        st = storage or self.storage
        # same LAPACK layout (leading dimension) when the storage kind and extent are kept
        lld = self.ld if (st == STORAGE_LAPACK and self.storage == STORAGE_LAPACK and lm is None) else None
        return TiledMatrix(dtype or self.dtype, self.mb, self.nb, lm or self.m, ln or self.n, P=self.grid.P,
                           Q=self.grid.Q, kp=self.grid.kp, kq=self.grid.kq, ip=self.grid.ip, jq=self.grid.jq,
                           rank=self.rank, device=self.device, storage=st, lld=lld,
                           uplo=self.uplo, alloc=alloc, name=name or self.name)

    # ------------------------------------------------------------ host helpers (tests / checks)
    def to_dense_local(self) -> torch.Tensor:
        """Assemble this rank's tiles into an m x n dense CPU tensor (zeros elsewhere)."""
        out = torch.zeros(self.m, self.n, dtype=self.dtype)
        for (m, n) in self.local_tiles():
            r0, c0 = m * self.mb, n * self.nb
            out[r0:r0 + self.tile_rows(m), c0:c0 + self.tile_cols(n)] = self.tile(m, n).cpu()
        return out

    def from_dense(self, M: torch.Tensor):
        """Scatter a dense m x n tensor into the local tiles."""
        for (m, n) in self.local_tiles():
            r0, c0 = m * self.mb, n * self.nb
            self.tile(m, n).copy_(M[r0:r0 + self.tile_rows(m), c0:c0 + self.tile_cols(n)].to(self.device))
        return self

    def __repr__(self):
        return (f"TiledMatrix({self.name}, {self.prec}, {self.m}x{self.n} mb={self.mb} nb={self.nb} "
                f"grid={self.grid.P}x{self.grid.Q} rank={self.rank} {self.storage} dev={self.device})")


def block_cyclic(ctx, dtype, mb, nb, m, n, *, storage=STORAGE_TILE, kp=1, kq=1, ip=0, jq=0, lld=None,
                 uplo=dplasmaUpperLower, name="A", alloc=True) -> TiledMatrix:
    """Allocate a descriptor distributed on the context's process grid."""
    return TiledMatrix(dtype, mb, nb, m, n, P=ctx.P, Q=ctx.Q, kp=kp, kq=kq, ip=ip, jq=jq, rank=ctx.rank,
                       device=ctx.device, storage=storage, lld=lld, uplo=uplo, name=name, alloc=alloc)


def sym_block_cyclic(ctx, dtype, mb, nb, n, uplo, **kw) -> TiledMatrix:
    """Symmetric/Hermitian matrix descriptor (only ``uplo`` triangle is referenced)."""
    return block_cyclic(ctx, dtype, mb, nb, n, n, uplo=uplo, **kw)
