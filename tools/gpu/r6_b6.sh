#!/bin/bash
# r6 batch 6: kernel trace of one LU replay rank (2x4 64k, gather panel, p2p interchanges, look-ahead)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b6
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
echo "== rocprofv3 kernel trace, replay rank 0 (gather)" | tee -a $O/summary.log
DPLASMA_LU_PANEL=gather timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o rank0 -- \
  python tools/replay_lu.py -N 65536 --nb 512 --grid 2x4 --ranks 0 --xlat 3.3 --xgmi 2 > $O/rp.log 2>&1 \
  || { tail -30 $O/rp.log | tee -a $O/summary.log; exit 1; }
grep -E "^rank" $O/rp.log | tee -a $O/summary.log
find $O/tr -name "*kernel_trace.csv" | head -3 | tee -a $O/summary.log
echo "== DTR probe v3 (POTRF input snapshot), queue, 512 WGs, 32k x 30" | tee -a $O/summary.log
DPLASMA_DTR_PROBE=1 DPLASMA_DTR_SNAP=1 DPLASMA_DTR_WG=512 timeout -k 10 500 python tools/gpu/dtr_repeat.py 32768 30 \
  > $O/probe.log 2>&1 || { tail -20 $O/probe.log | tee -a $O/summary.log; exit 1; }
grep -E "check=False|FAILED" $O/probe.log | sed -e 's/first (j, i, r, c, err): \[[^]]*\]//' | cut -c1-600 | tail -12 | tee -a $O/summary.log
exit 0
