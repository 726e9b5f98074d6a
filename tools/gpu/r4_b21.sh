#!/bin/bash
# r4 batch 21: LU-QR / getrf_1d with the 32-column (64 KiB LDS) pivoting block kernel, which leaves room on a CU
# for a trailing-update GEMM workgroup beside it; POTRF auto engine (dtr window 24k..48k) sanity;
# QR panel: T-coupling Z on MFMA, replica update loads before stores.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r4b21
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|error|Error|TF/s|TIME|gflops|wall" $O/$name.log | grep -v amdgpu.ids | tail -6 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step qr_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_qr.py -m gpu || exit 1
step panel_prof 120 python tools/gpu/qr_panel_prof.py 256 1024 32768 || exit 1
step luqr_bw32 300 env DPLASMA_LU_BW=32 python tools/gpu/luqr_syncdebug.py 32768 256 || exit 1
step luqr_lu_only_bw32 300 env DPLASMA_LU_BW=32 python tools/gpu/luqr_syncdebug.py 32768 256 3 || exit 1
step getrf32k_la_bw32 200 env DPLASMA_LU_BW=32 DPLASMA_LU_LOOKAHEAD=1 python tools/bench_algo.py getrf_1d -N 32768 --nb 512 --runs 2 || exit 1
step getrf32k_base 200 python tools/bench_algo.py getrf_1d -N 32768 --nb 512 --runs 2 || exit 1
step getrf64k_la_bw32 300 env DPLASMA_LU_BW=32 DPLASMA_LU_LOOKAHEAD=1 python tools/bench_algo.py getrf_1d -N 65536 --nb 512 --runs 1 || exit 1
step potrf_auto 300 python -m dplasma_amd.testing dpotrf -N 32768 -t 512 -x || exit 1
exit 0
