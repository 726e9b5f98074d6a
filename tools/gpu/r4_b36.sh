#!/bin/bash
# r4 batch 36: the C ABI GPU tests (native one-process and grid contexts, F77 shims) on the final library, and smoke
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4b36
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|FAIL|smoke" $O/$name.log | grep -v amdgpu.ids | tail -6 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step capi_gpu 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_capi.py -m gpu || exit 1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
exit 0
