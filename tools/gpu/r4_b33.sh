#!/bin/bash
# r4 batch 33: native C ABI additions (geru / gerc, laswp, lanm2, trsmpl_ptgpanel, trsmpl_incpiv, trdsm, trmdm, hetrf, hetrs, print) and the getrs swap refactor under the native tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4b33
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|error|Error|FAIL|dgeru|zgerc|dlaswp|dlanm2|dpltmg|hebut|dtrsmpl|dtrdsm|dtrmdm|hetrf|incpiv|A\(|dgetrs|dgesv|native C ABI" $O/$name.log | grep -v amdgpu.ids | tail -12 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
gcc -O2 -o $O/test_native tests/capi/test_native.c -Icapi/include -Ldplasma_amd/lib -ldplasma -lm \
  -Wl,-rpath,$PWD/dplasma_amd/lib || exit 1
step native_bin 300 $O/test_native || exit 1
rm -f $O/test_native
exit 0
