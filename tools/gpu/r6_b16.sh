#!/bin/bash
# r6 batch 16: HQR config 4 rank replay (2x4 64k NB=256, all ranks) after the panel T_b / reduction changes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b16
mkdir -p $O
export PYTHONUNBUFFERED=1
echo "== HQR replay 2x4 64k" | tee -a $O/summary.log
GPU_MAX_HW_QUEUES=16 timeout -k 10 900 python tools/replay_hqr.py -N 65536 --nb 256 --grid 2x4 --bw 65 --lat 10 \
  > $O/rp.log 2>&1 || { tail -30 $O/rp.log | tee -a $O/summary.log; exit 1; }
grep -E "^rank|pct_peak" $O/rp.log | tee -a $O/summary.log
exit 0
