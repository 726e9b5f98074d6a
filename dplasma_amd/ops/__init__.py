"""Tile kernels: batched HIP/CDNA4 launches (GPU) and CPU reference kernels."""
from . import tile_ops  # noqa: F401
from .batch import GemmBatch, TileBatch  # noqa: F401
