#!/bin/bash
# r4 batch 32: native C ABI additions (geru / gerc, laswp, lanm2, trsmpl_ptgpanel, trsmpl_incpiv, trdsm, trmdm, hetrf, hetrs, print) and the getrs swap refactor under the native tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4b32
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|error|Error|FAIL|dgeru|zgerc|dlaswp|dlanm2|dtrsmpl|dtrdsm|dtrmdm|hetrf|incpiv|A\(|dgetrs|dgesv|native C ABI" $O/$name.log | grep -v amdgpu.ids | tail -12 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step capi_gpu 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_capi.py -m gpu || exit 1
gcc -O2 -o $O/test_native tests/capi/test_native.c -Icapi/include -Ldplasma_amd/lib -ldplasma -lm \
  -Wl,-rpath,$PWD/dplasma_amd/lib || exit 1
step native_bin 300 $O/test_native || exit 1
rm -f $O/test_native
step gpu_suite 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench 400 python bench.py --steps 20 --warmup 5 || exit 1
grep -E '^\{' $O/bench.log | cut -c1-400
exit 0
