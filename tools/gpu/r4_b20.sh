#!/bin/bash
# r4 batch 20: where LU-QR's time goes -- LU-only / QR-only criteria, getrf_1d at NB=256, kernel split of DEFAULT.
# (rerun after the fix of the first attempt's fault: the LU engine's single panel buffer under LU-QR look-ahead)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r4b20
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|error|Error|TF/s|TIME" $O/$name.log | grep -v amdgpu.ids | tail -6 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step luqr_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lu_qr.py -m gpu || exit 1
step luqr_lu_only 300 python tools/gpu/luqr_syncdebug.py 32768 256 3 || exit 1
step luqr_qr_only 300 python tools/gpu/luqr_syncdebug.py 32768 256 4 || exit 1
step getrf32k_nb256 200 python tools/bench_algo.py getrf_1d -N 32768 --nb 256 --runs 2 || exit 1
cd /tmp && export TMPDIR=/tmp
step luqr_prof 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o luqr -- python3 $R/tools/gpu/luqr_syncdebug.py 32768 256 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -14 "$f" | cut -c1-150 | tee -a $O/summary.log
exit 0
