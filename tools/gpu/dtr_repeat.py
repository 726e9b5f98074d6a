"""Repeat one DTR Cholesky configuration and residual-check every run (intermittent-failure hunt).

  python tools/gpu/dtr_repeat.py N runs
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402

import dplasma_amd as dp  # noqa: E402
from dplasma_amd.models import potrf_dtr as D  # noqa: E402


def main():
    N, runs = int(sys.argv[1]), int(sys.argv[2])
    ctx = dp.init()
    A = dp.block_cyclic(ctx, torch.float64, 512, 512, N, N)
    dp.dplghe(ctx, float(N), dp.dplasmaLower, A, 3872)
    A0 = A.data.clone()
    tp = D.potrf_dtr_New(ctx, dp.dplasmaLower, A)
    Ar = A.like()
    bad = 0
    for rep in range(runs):
        A.data.copy_(A0)
        tp.info.zero_()
        tp.execute(ctx)
        Ar.data.copy_(A0)
        ok, res = dp.check_potrf(ctx, dp.dplasmaLower, A, Ar)
        bad += not ok
        print(f"run {rep}: check={ok} res={res:.2e}", flush=True)
    print(f"FAILED {bad} / {runs}", flush=True)


if __name__ == "__main__":
    main()
