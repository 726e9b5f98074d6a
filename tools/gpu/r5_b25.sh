#!/bin/bash
# r5 batch 25: step-order failure under the long hold with write-through update/TRSM results; perf of 256 vs 512 WGs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b25
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {
  local name=$1; shift
  echo "== $name" | tee -a $O/summary.log
  env DPLASMA_DTR_LO_ORDER=step DPLASMA_DTR_STEPW=2 DPLASMA_DTR_HOLD=2550,0 "$@" timeout -k 10 300 python tools/gpu/dtr_repeat.py 32768 30 > $O/$name.log 2>&1
  local rc=$?
  grep -E "False|FAILED" $O/$name.log | cut -c1-300 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
run wt DPLASMA_DTR_WT=1 || exit 1
echo "== perf column 512 WGs" | tee -a $O/summary.log
timeout -k 10 300 python tools/gpu/dtr_bench.py 16384 32768 65536 2>&1 | grep TIME | tee -a $O/summary.log
echo "== perf column 256 WGs" | tee -a $O/summary.log
DPLASMA_DTR_WG=256 timeout -k 10 200 python -c "
import sys; sys.path.insert(0, 'tools/gpu'); import dtr_bench as b
for N in (16384, 32768, 65536): b.run(N, 'dtr')" 2>&1 | grep TIME | tee -a $O/summary.log
exit 0
