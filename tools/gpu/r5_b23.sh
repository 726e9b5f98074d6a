#!/bin/bash
# r5 batch 23: POTRF tile input through L1-bypassing loads -- step-order failure under the long hold; column under hold
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b23
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {
  local name=$1; shift
  echo "== $name" | tee -a $O/summary.log
  env DPLASMA_DTR_HOLD=2550,0 "$@" timeout -k 10 300 python tools/gpu/dtr_repeat.py 32768 30 > $O/$name.log 2>&1
  local rc=$?
  grep -E "False|FAILED" $O/$name.log | cut -c1-300 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
run step_w2 DPLASMA_DTR_LO_ORDER=step DPLASMA_DTR_STEPW=2 || exit 1
run column DPLASMA_DTR_LO_ORDER=column || exit 1
exit 0
