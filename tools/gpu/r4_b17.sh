#!/bin/bash
# r4 batch 17: HQR on one process row -- TT subtree of a step as ONE stacked panel of triangles, batched
# look-ahead, Gram-downdated panel column steps.  QR/LU-QR GPU tests, panel timers on fresh data,
# flat / HQR a=4 / a=16 at 32k, HQR a=16 at 64k, LU-QR 32k under sync-debug.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r4b17
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|error|Error|TF/s|TIME|wall|columns" $O/$name.log | grep -v amdgpu.ids | tail -14 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step qr_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_qr.py tests/test_lu_qr.py -m gpu || exit 1
step panel_prof 120 python tools/gpu/qr_panel_prof.py 256 1024 4096 8192 32768 || exit 1
step hqr32k_a4 200 python tools/bench_algo.py geqrf -N 32768 --nb 256 --ib 32 --runs 2 --tree hqr --qr-llvl 1 --qr-hlvl 0 --qr-a 4 || exit 1
step hqr32k_a16 200 python tools/bench_algo.py geqrf -N 32768 --nb 256 --ib 32 --runs 2 --tree hqr --qr-llvl 1 --qr-hlvl 0 --qr-a 16 || exit 1
step geqrf32k_flat 200 python tools/bench_algo.py geqrf -N 32768 --nb 256 --ib 32 --runs 2 || exit 1
step hqr64k_a16 300 python tools/bench_algo.py geqrf -N 65536 --nb 256 --ib 32 --runs 1 --tree hqr --qr-llvl 1 --qr-hlvl 0 --qr-a 16 || exit 1
step luqr_sync32k 400 python tools/gpu/luqr_syncdebug.py 32768 256 || exit 1
cd /tmp && export TMPDIR=/tmp
step hqr32k_prof 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o hqr -- python3 $R/tools/bench_algo.py geqrf -N 32768 --nb 256 --ib 32 --runs 1 --tree hqr --qr-llvl 1 --qr-hlvl 0 --qr-a 4 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -10 "$f" | cut -c1-150 | tee -a $O/summary.log
exit 0
