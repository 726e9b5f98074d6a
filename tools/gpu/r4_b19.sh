#!/bin/bash
# r4 batch 19: panel Y-partials / trailing prefetch + MFMA T^T Y; LU-QR look-ahead across LU and QR steps; HQR 2x4 replay with
# the Gram-downdated panel (cross-row TT kills stay pairwise).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r4b19
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|error|Error|TF/s|TIME|wall|columns|worst|rank .*ms" $O/$name.log | grep -v amdgpu.ids | tail -14 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step qr_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_qr.py tests/test_lu_qr.py -m gpu || exit 1
step panel_prof 120 python tools/gpu/qr_panel_prof.py 256 1024 8192 32768 || exit 1
step hqr32k_a4 200 python tools/bench_algo.py geqrf -N 32768 --nb 256 --ib 32 --runs 2 --tree hqr --qr-llvl 1 --qr-hlvl 0 --qr-a 4 || exit 1
step geqrf32k_flat 200 python tools/bench_algo.py geqrf -N 32768 --nb 256 --ib 32 --runs 2 || exit 1
step luqr_sync32k 400 python tools/gpu/luqr_syncdebug.py 32768 256 || exit 1
step luqr_cli8k 300 python -m dplasma_amd.testing dgetrf_qrf -N 8192 -t 256 -T 256 -x || exit 1
step hqr_replay_2x4 900 python tools/replay_hqr.py -N 65536 --nb 256 --grid 2x4 --ranks all --bw 65 --lat 10 || exit 1
exit 0
