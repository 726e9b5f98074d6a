#!/bin/bash
# r4 batch 29: DTR -- a workgroup whose own XCD list head is not ready steals a ready head of another XCD's list
# (DPLASMA_DTR_STEAL=1) vs the default (steal only from exhausted lists).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4b29
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|error|Error|TF/s|TIME|span=|occupancy|busy %" $O/$name.log | grep -v amdgpu.ids | tail -8 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step dtr_tests 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_potrf_dtr.py -m gpu || exit 1
step bench_base 300 python tools/gpu/dtr_bench.py 32768 65536 || exit 1
step bench_steal 300 env DPLASMA_DTR_STEAL=1 python tools/gpu/dtr_bench.py 32768 65536 || exit 1
step trace64k_steal 240 env DPLASMA_DTR_STEAL=1 python tools/gpu/dtr_trace_run.py 65536 || exit 1
exit 0
