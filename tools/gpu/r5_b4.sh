#!/bin/bash
# r5 batch 4: multi-rank DTR kernel -- single-rank regression (tests + 16k/32k perf), grid emulation
# correctness (residual) and the first modelled P x Q times
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b4
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|FAIL|Error|error|TIME|EMUL|emul\]|residual" $O/$name.log | grep -v amdgpu.ids | tail -14 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step tests 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_potrf_dtr.py || exit 1
step perf 300 python tools/gpu/dtr_bench.py 16384 32768 || exit 1
step em16_1x2 200 python tools/emulate_potrf.py -N 16384 --grid 1x2 --check || exit 1
step em16_2x4 200 python tools/emulate_potrf.py -N 16384 --grid 2x4 --check || exit 1
step em32_2x4 300 python tools/emulate_potrf.py -N 32768 --grid 2x4 --check || exit 1
step em64_2x4 400 python tools/emulate_potrf.py -N 65536 --grid 2x4 --reps 1 || exit 1
exit 0
