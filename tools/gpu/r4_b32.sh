#!/bin/bash
# r4 batch 32: native C ABI additions (geru / gerc, laswp, lanm2) and the getrs swap refactor under the native tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4b32
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|error|Error|FAIL|dgeru|zgerc|dlaswp|dlanm2|dgetrs|dgesv" $O/$name.log | grep -v amdgpu.ids | tail -12 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step capi_gpu 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_capi.py -m gpu || exit 1
exit 0
