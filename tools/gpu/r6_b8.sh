#!/bin/bash
# r6 batch 8: DTR POTRF-task fault localisation (32 x 32 blocks of the wrong diagonal factor) + 2x4 LU rehearsals
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b8
mkdir -p $O
export PYTHONUNBUFFERED=1
echo "== DTR probe v4, queue, 512 WGs, 32k x 30" | tee -a $O/summary.log
DPLASMA_DTR_PROBE=1 DPLASMA_DTR_SNAP=1 DPLASMA_DTR_WG=512 timeout -k 10 500 python tools/gpu/dtr_repeat.py 32768 30 \
  > $O/probe.log 2>&1 || { tail -20 $O/probe.log | tee -a $O/summary.log; exit 1; }
grep -E "check=False|FAILED" $O/probe.log | sed -e 's/first (j, i, r, c, err): \[[^]]*\]//' -e 's/counters off.*//' | cut -c1-900 | tail -12 | tee -a $O/summary.log
echo "== 2x4 LU grid rehearsals (8 processes, one GPU)" | tee -a $O/summary.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_lu_dist.py -m gpu -x -v --timeout 420 --timeout-method thread -k 2x4 \
  > $O/lu2x4.log 2>&1; rc=$?
grep -E "PASS|FAIL|passed|failed|SUCCESS" $O/lu2x4.log | cut -c1-300 | tail -20 | tee -a $O/summary.log
exit $rc
