#!/bin/bash
# r5 batch 20: segmented step order failure -- system-scope release / long POTRF ticket hold / one workgroup per CU
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b20
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {
  local name=$1; shift
  echo "== $name" | tee -a $O/summary.log
  env DPLASMA_DTR_LO_ORDER=step DPLASMA_DTR_STEPW=2 "$@" timeout -k 10 300 python tools/gpu/dtr_repeat.py 32768 30 > $O/$name.log 2>&1
  local rc=$?
  grep -E "False|FAILED" $O/$name.log | cut -c1-400 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
run sysrel DPLASMA_DTR_SYSREL=1 || exit 1
run hold DPLASMA_DTR_HOLD=2550,0 || exit 1
run wg256 DPLASMA_DTR_WG=256 || exit 1
exit 0
