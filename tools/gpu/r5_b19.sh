#!/bin/bash
# r5 batch 19: localise the segmented step order's intermittent wrong factor (wrong 128x128 sub-tiles vs a good run)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b19
mkdir -p $O
export PYTHONUNBUFFERED=1
echo "== step_w2 32k" | tee -a $O/summary.log
DPLASMA_DTR_LO_ORDER=step DPLASMA_DTR_STEPW=2 timeout -k 10 400 python tools/gpu/dtr_repeat.py 32768 20 > $O/step_w2.log 2>&1
echo "rc=$?" | tee -a $O/summary.log
grep -E "False|FAILED" $O/step_w2.log | tee -a $O/summary.log
exit 0
