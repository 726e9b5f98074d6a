"""dplasma_amd -- MI355X-native distributed tile dense linear algebra.

Same capabilities and API shape as DPLASMA (``src/include/dplasma/dplasma_z.h``):
every operation ``op`` exists as a blocking call ``op(ctx, ...)``, a taskpool
constructor ``op_New(ctx, ...)`` and ``op_Destruct(tp)``, plus precision-prefixed
aliases (``dpotrf``, ``zgemm``, ...).  Matrices are 2-D block-cyclic tiled
descriptors (``descriptor.TiledMatrix``) living in HBM, one process per GPU.

Layout:
  ops/       HIP/CDNA4 tile kernels (batched) + CPU reference tile kernels
  models/    algorithm families (Cholesky, LU, QR, BLAS3, norms, generators ...)
  parallel/  process grid communication (RCCL/xGMI via torch.distributed)
  runtime/   taskpools, stream-program executor, tile DAGs (native level analysis), DTD
  utils/     flops, LCG generators, options, tracing
"""
from .constants import *  # noqa: F401,F403
from .context import Context, fini, init  # noqa: F401
from .descriptor import Grid, TiledMatrix, block_cyclic, sym_block_cyclic  # noqa: F401
from . import api  # noqa: F401
from .api import *  # noqa: F401,F403

__version__ = "0.1.0"
