#!/bin/bash
# DGETRF block width 64 vs 32 (the 32-wide block kernel can share CUs with GEMM) x look-ahead; LU-QR profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_capi.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/b9_capi.log 2>&1
rc=$?; grep -E "passed|failed|FAIL" gpurun_out/b9_capi.log | tail -8; echo "capi rc=$rc"; [ $rc -ne 0 ] && exit $rc
for N in 32768 65536; do for BW in 64 32; do for LA in 0 1; do
  DPLASMA_LU_BW=$BW DPLASMA_LU_LOOKAHEAD=$LA timeout -k 10 200 python tools/bench_algo.py getrf_1d -N $N --nb 512 --runs 2 \
      > gpurun_out/b9_lu_${N}_${BW}_${LA}.log 2>&1 || { echo "lu $N $BW $LA failed"; tail -5 gpurun_out/b9_lu_${N}_${BW}_${LA}.log; exit 1; }
  echo "N=$N bw=$BW lookahead=$LA: $(grep TIME gpurun_out/b9_lu_${N}_${BW}_${LA}.log | tail -1 | cut -c1-150)"
done; done; done
timeout -k 10 400 python -u -m pytest tests/test_qr.py tests/test_api_variants.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/b9_qr.log 2>&1
rc=$?; tail -1 gpurun_out/b9_qr.log; echo "qr tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/replay_hqr.py -N 65536 --nb 256 --grid 2x4 --ranks 0,4 --steps 1 --bw 65 --lat 10 \
    > gpurun_out/b9_replay_hqr.log 2>&1
rc=$?; tail -3 gpurun_out/b9_replay_hqr.log | cut -c1-300; echo "replay hqr rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/gpu/luqr_prof.py 32768 256 > gpurun_out/b9_luqr_prof.log 2>&1
rc=$?; grep "^run" gpurun_out/b9_luqr_prof.log | cut -c1-40; echo "luqr rc=$rc"
exit 0
