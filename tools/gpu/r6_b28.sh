#!/bin/bash
# r6 batch 28: DGETRF one GPU -- deferred left interchanges (DPLASMA_LU_DEFER_LEFT): bitwise parity on the GPU, then
# 32k / 64k against the per-step moves
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b28
mkdir -p $O
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
timeout -k 10 200 python - <<'PY' 2>&1 | tee $O/parity.log
import os, torch
import dplasma_amd as dp
ctx = dp.init(device="cuda:0")
for (M, N) in [(8192, 8192), (9000, 6000)]:
    out = []
    for mode in ("0", "1"):
        os.environ["DPLASMA_LU_DEFER_LEFT"] = mode
        A = dp.block_cyclic(ctx, torch.float64, 512, 512, M, N)
        dp.plrnt(ctx, A, 3872)
        IP = dp.ipiv_descriptor(ctx, A)
        tp = dp.getrf_1d_New(ctx, A, IP)
        tp.execute(ctx)
        torch.cuda.synchronize()
        out.append((A.to_dense_local().cpu(), IP.to_dense_local().cpu(), tp._state.defer_left))
    print(f"M={M} N={N} defer={out[1][2]} factors identical={torch.equal(out[0][0], out[1][0])} "
          f"pivots identical={torch.equal(out[0][1], out[1][1])}", flush=True)
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
PY
[ ${PIPESTATUS[0]} -eq 0 ] || exit 1
for N in 32768 65536; do
  for m in 0 1 0 1; do
    echo "== N=$N DEFER_LEFT=$m" | tee -a $O/summary.log
    DPLASMA_LU_DEFER_LEFT=$m timeout -k 10 240 python tools/bench_algo.py getrf_1d -N $N --nb 512 --runs 2 > $O/${N}_$m.log 2>&1 || { tail -5 $O/${N}_$m.log; exit 1; }
    grep TIME $O/${N}_$m.log | tail -1 | cut -c1-140 | tee -a $O/summary.log
  done
done
exit 0
