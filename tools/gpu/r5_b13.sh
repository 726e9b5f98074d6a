#!/bin/bash
# r5 batch 13: intermittent wrong factor -- repeated residual-checked 32k runs: column order (control), step order
# with one segment scanned (single FIFO), step order with 8 segments
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b13
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {
  local name=$1; shift
  echo "== $name" | tee -a $O/summary.log
  env "$@" timeout -k 10 300 python tools/gpu/dtr_repeat.py 32768 12 > $O/$name.log 2>&1
  local rc=$?
  grep -E "FAILED|False" $O/$name.log | tail -4 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
run column DPLASMA_DTR_LO_ORDER=column || exit 1
run step_w1 DPLASMA_DTR_LO_ORDER=step DPLASMA_DTR_STEPW=1 || exit 1
run step_w8 DPLASMA_DTR_LO_ORDER=step DPLASMA_DTR_STEPW=8 || exit 1
run step_w2 DPLASMA_DTR_LO_ORDER=step DPLASMA_DTR_STEPW=2 || exit 1
exit 0
