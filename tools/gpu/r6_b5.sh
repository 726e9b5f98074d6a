#!/bin/bash
# r6 batch 5: DTR hazard probe v2 (strip stamps + diagonal sub-tile version stamps + POTRF input), 512 workgroups
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b5
mkdir -p $O
export PYTHONUNBUFFERED=1
echo "== DTR probe v2, queue scheduler, 512 WGs, 32k x 30" | tee -a $O/summary.log
DPLASMA_DTR_PROBE=1 DPLASMA_DTR_WG=512 timeout -k 10 400 python tools/gpu/dtr_repeat.py 32768 30 > $O/probe.log 2>&1 \
  || { tail -20 $O/probe.log | tee -a $O/summary.log; exit 1; }
grep -E "check=False|probe:|FAILED" $O/probe.log | cut -c1-900 | tail -14 | tee -a $O/summary.log
exit 0
