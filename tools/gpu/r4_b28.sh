#!/bin/bash
# r4 batch 28: where DGETRF 64k spends its time (kernel split), plus the row-move hardening under the LU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r4b28
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|error|Error|TF/s|TIME" $O/$name.log | grep -v amdgpu.ids | tail -4 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step lu_tests 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_lu.py tests/test_gpu_lu_dist.py -m gpu || exit 1
cd /tmp && export TMPDIR=/tmp
step getrf64k_prof 400 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o lu -- python3 $R/tools/bench_algo.py getrf_1d -N 65536 --nb 512 --runs 1 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -16 "$f" | cut -c1-150 | tee -a $O/summary.log
exit 0
