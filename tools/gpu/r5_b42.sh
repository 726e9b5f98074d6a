#!/bin/bash
# r5 batch 42: correctness of the push-scheduled DTR under the adopted bottom-level weights (400 / 800):
# repeated residual-checked runs at 16k / 32k, the emulated 2x4 grid at 32k with its factor checked, DTR GPU tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b42
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|rror|bad|ok|EMUL|residual|runs" $O/$name.log | grep -v amdgpu.ids | tail -8 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step dtr_tests 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_potrf_dtr.py -m gpu || exit 1
step rep16k 200 python tools/gpu/dtr_repeat.py 16384 16 || exit 1
step rep32k 300 python tools/gpu/dtr_repeat.py 32768 12 || exit 1
step emul32k 300 env DPLASMA_DTR_WG=256 python tools/emulate_potrf.py -N 32768 --grid 2x4 --bw 50 --lat 10 --reps 1 --check || exit 1
exit 0
