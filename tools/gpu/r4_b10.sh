#!/bin/bash
# r4 batch 10: QR panel kernel (MFMA T coupling, one-workgroup shortcuts): QR / HQR / LU-QR GPU tests, then
# flat and HQR DGEQRF timings and the device-resident LU-QR at 32k.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4b10
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|error|Error|TF/s|TIME|span=|occupancy|worst|pct_peak" $O/$name.log | grep -v amdgpu.ids | tail -6 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step dtr_tests 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_potrf_dtr.py -m gpu || exit 1
step dtr_bench 400 python tools/gpu/dtr_bench.py 16384 32768 65536 || exit 1
step dtr_trace64k 200 python tools/gpu/dtr_trace_run.py 65536 $O/dtr64k.npz || exit 1
step qr_tests 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_qr.py tests/test_lu_qr.py -m gpu || exit 1
step geqrf32k_flat 200 python tools/bench_algo.py geqrf -N 32768 --nb 256 --ib 32 --runs 2 || exit 1
step hqr32k_a4 300 python tools/bench_algo.py geqrf -N 32768 --nb 256 --ib 32 --runs 2 --tree hqr --qr-llvl 1 --qr-hlvl 0 --qr-a -1 || exit 1
step hqr32k_a16 300 python tools/bench_algo.py geqrf -N 32768 --nb 256 --ib 32 --runs 2 --tree hqr --qr-llvl 1 --qr-hlvl 0 --qr-a 16 || exit 1
step luqr_sync32k 400 python tools/gpu/luqr_syncdebug.py 32768 256 || exit 1
exit 0
