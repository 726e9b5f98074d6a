#!/bin/bash
# r4 batch 14: DTR with the bulk updates assigned to XCDs by tile row (gaps at 64k, benches); native C tests
# (incremental-pivoting LU added).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4b14
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|error|Error|TF/s|TIME|span=|occupancy|gaps|next task|busy %" $O/$name.log | grep -v amdgpu.ids | tail -14 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step dtr_tests 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_potrf_dtr.py -m gpu || exit 1
step dtr_trace64k 240 python tools/gpu/dtr_trace_run.py 65536 || exit 1
step dtr_bench 500 python tools/gpu/dtr_bench.py 16384 32768 65536 || exit 1
step dtr_bench_D6 300 env DPLASMA_DTR_DEFER=6 python tools/gpu/dtr_bench.py 65536 || exit 1
step capi_native 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_capi.py -m gpu -k "native_gpu" || exit 1
exit 0
