#!/bin/bash
# r5 batch 3: DTR ticket-hold policy sweep (DPLASMA_DTR_HOLD="potrf_us,other_us") at 16k / 32k, with a trace at 16k
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b3
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "TIME|span|occupancy|POTRF|TRSM|UPD" $O/$name.log | head -14 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
run base 300 python tools/gpu/dtr_bench.py 16384 32768 || exit 1
for h in "50,0" "500,0" "500,100" "500,500" "2000,2000"; do
  DPLASMA_DTR_HOLD=$h run "hold_${h/,/_}" 300 python -c "
import sys; sys.path.insert(0, 'tools/gpu'); import dtr_bench as b
for N in (16384, 32768): b.run(N, 'dtr')" || exit 1
done
run trace16k 300 python tools/gpu/dtr_trace_run.py 16384 || exit 1
exit 0
