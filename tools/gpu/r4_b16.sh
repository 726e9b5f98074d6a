#!/bin/bash
# r4 batch 16: Gram-downdated QR panel column steps (QR tests, panel phase timers, flat + HQR a=4 32k, kernel split);
# DTR after reverting the combined peek (64k vs stream).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r4b16
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|error|Error|TF/s|TIME|span=|occupancy|wall" $O/$name.log | grep -v amdgpu.ids | tail -14 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step qr_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_qr.py tests/test_lu_qr.py -m gpu || exit 1
step panel_prof 120 python tools/gpu/qr_panel_prof.py 256 512 1024 4096 32768 || exit 1
step geqrf32k_flat 200 python tools/bench_algo.py geqrf -N 32768 --nb 256 --ib 32 --runs 2 || exit 1
step dtr_tests 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_potrf_dtr.py -m gpu || exit 1
step dtr_bench 300 python tools/gpu/dtr_bench.py 65536 || exit 1
cd /tmp && export TMPDIR=/tmp
step hqr32k_prof 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o hqr -- python3 $R/tools/bench_algo.py geqrf -N 32768 --nb 256 --ib 32 --runs 1 --tree hqr --qr-llvl 1 --qr-hlvl 0 --qr-a -1 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -14 "$f" | cut -c1-160 | tee -a $O/summary.log
exit 0
