#!/bin/bash
# r5 batch 2: native C ABI after the pivot-info fix; the stream-priority probe cited by dtr.hip; short bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b2
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|FAIL|TIME|corrupt|ms|GFLOP" $O/$name.log | grep -v amdgpu.ids | tail -14 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
step capi 600 $T tests/test_capi.py tests/test_pivot_guard.py || exit 1
step prio 300 python tools/gpu/prio_probe.py 96 2 0 512 || exit 1
step bench 300 python bench.py --steps 3 --warmup 1 || exit 1
exit 0
