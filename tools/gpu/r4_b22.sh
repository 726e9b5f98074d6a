#!/bin/bash
# r4 batch 22: HQR / LU-QR with Y = V T^T formed once per reflector set (C -= Y (V^T C), no T^T W product);
# getrf_1d NB=256 with look-ahead and the 32-column pivoting block.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r4b22
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|error|Error|TF/s|TIME|gflops" $O/$name.log | grep -v amdgpu.ids | tail -6 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step qr_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_qr.py tests/test_lu_qr.py -m gpu || exit 1
step hqr32k_a4 200 python tools/bench_algo.py geqrf -N 32768 --nb 256 --ib 32 --runs 2 --tree hqr --qr-llvl 1 --qr-hlvl 0 --qr-a 4 || exit 1
step hqr32k_a16 200 python tools/bench_algo.py geqrf -N 32768 --nb 256 --ib 32 --runs 2 --tree hqr --qr-llvl 1 --qr-hlvl 0 --qr-a 16 || exit 1
step luqr32k 300 python tools/gpu/luqr_syncdebug.py 32768 256 || exit 1
step luqr32k_bw32 300 env DPLASMA_LU_BW=32 python tools/gpu/luqr_syncdebug.py 32768 256 || exit 1
step getrf32k_nb256_la_bw32 200 env DPLASMA_LU_BW=32 DPLASMA_LU_LOOKAHEAD=1 python tools/bench_algo.py getrf_1d -N 32768 --nb 256 --runs 2 || exit 1
step getrf64k_nb256_la_bw32 300 env DPLASMA_LU_BW=32 DPLASMA_LU_LOOKAHEAD=1 python tools/bench_algo.py getrf_1d -N 65536 --nb 256 --runs 1 || exit 1
exit 0
