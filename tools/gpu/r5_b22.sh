#!/bin/bash
# r5 batch 22: the step-order failure under the long POTRF ticket hold (~20 % of runs) -- which knob removes it
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b22
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
run sysrel DPLASMA_DTR_SYSREL=1 || exit 1
run sysacq DPLASMA_DTR_SYSACQ=1 || exit 1
run wg256 DPLASMA_DTR_WG=256 || exit 1
exit 0
