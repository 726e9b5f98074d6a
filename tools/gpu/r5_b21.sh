#!/bin/bash
# r5 batch 21: system-scope release for diagonal sub-tile updates only -- step order failure rate; column perf
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b21
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {
  local name=$1; shift
  echo "== $name" | tee -a $O/summary.log
  env "$@" timeout -k 10 300 python tools/gpu/dtr_repeat.py 32768 30 > $O/$name.log 2>&1
  local rc=$?
  grep -E "False|FAILED" $O/$name.log | cut -c1-400 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
run step_w2_hold DPLASMA_DTR_LO_ORDER=step DPLASMA_DTR_STEPW=2 DPLASMA_DTR_HOLD=2550,0 || exit 1
run step_w8 DPLASMA_DTR_LO_ORDER=step DPLASMA_DTR_STEPW=8 || exit 1
echo "== perf column" | tee -a $O/summary.log
timeout -k 10 300 python tools/gpu/dtr_bench.py 16384 32768 65536 2>&1 | grep TIME | tee -a $O/summary.log
echo "== perf step w8" | tee -a $O/summary.log
DPLASMA_DTR_LO_ORDER=step DPLASMA_DTR_STEPW=8 timeout -k 10 200 python -c "
import sys; sys.path.insert(0, 'tools/gpu'); import dtr_bench as b
for N in (16384, 32768, 65536): b.run(N, 'dtr')" 2>&1 | grep TIME | tee -a $O/summary.log
exit 0
