#!/bin/bash
# r5 batch 14: (1) the intermittent DTR wrong-factor hunt (repeated residual-checked 32k runs: column control,
# step order with 1 / 8 segments scanned); (2) the config-5 model: getrf_ptgpanel 2x4 N=65536 rank replay with
# the true pivots delivered by the modelled broadcasts
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b14
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {
  local name=$1; shift
  echo "== $name" | tee -a $O/summary.log
  env "$@" timeout -k 10 300 python tools/gpu/dtr_repeat.py 32768 10 > $O/$name.log 2>&1
  local rc=$?
  grep -E "FAILED|False" $O/$name.log | tail -4 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
run column DPLASMA_DTR_LO_ORDER=column || exit 1
run step_w1 DPLASMA_DTR_LO_ORDER=step DPLASMA_DTR_STEPW=1 || exit 1
run step_w8 DPLASMA_DTR_LO_ORDER=step DPLASMA_DTR_STEPW=8 || exit 1
echo "== lu_replay" | tee -a $O/summary.log
timeout -k 10 900 python tools/replay_lu.py -N 65536 --nb 512 --grid 2x4 --bw 50 --lat 15 > $O/lu_replay.log 2>&1
echo "rc=$?" | tee -a $O/summary.log
grep -E "true pivots|rank |pct_peak" $O/lu_replay.log | tee -a $O/summary.log
exit 0
