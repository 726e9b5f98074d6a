#!/bin/bash
# r5 batch 26: step-order failure under the long hold -- are the counters at their final values after a failing run?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b26
mkdir -p $O
export PYTHONUNBUFFERED=1
echo "== step_w2_hold" | tee -a $O/summary.log
DPLASMA_DTR_LO_ORDER=step DPLASMA_DTR_STEPW=2 DPLASMA_DTR_HOLD=2550,0 timeout -k 10 300 python tools/gpu/dtr_repeat.py 32768 30 > $O/run.log 2>&1
echo "rc=$?" | tee -a $O/summary.log
grep -E "False|FAILED|counters" $O/run.log | cut -c1-600 | tee -a $O/summary.log
exit 0
