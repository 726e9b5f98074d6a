#!/bin/bash
# r6 batch 10: do the other rank replays serialise transfers on shared hardware queues?  HQR (config 4) and POTRF
# 2x4 64k rank replays with HIP's default 4 hardware queues per process vs 16
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b10
mkdir -p $O
export PYTHONUNBUFFERED=1
for q in 4 16; do
  echo "== HQR replay 2x4 64k NB=256 a=0, ranks 0,4, hw queues $q" | tee -a $O/summary.log
  GPU_MAX_HW_QUEUES=$q timeout -k 10 500 python tools/replay_hqr.py -N 65536 --nb 256 --grid 2x4 --ranks 0,4 --bw 65 --lat 10 \
    > $O/hqr_q$q.log 2>&1 || { tail -20 $O/hqr_q$q.log | tee -a $O/summary.log; exit 1; }
  grep -E "^rank|pct" $O/hqr_q$q.log | cut -c1-300 | tee -a $O/summary.log
  echo "== POTRF replay 2x4 64k, ranks 0,4, hw queues $q" | tee -a $O/summary.log
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python tools/replay_potrf.py -N 65536 --nb 512 --grid 2x4 --ranks 0,4 --steps 1 \
    > $O/potrf_q$q.log 2>&1 || { tail -20 $O/potrf_q$q.log | tee -a $O/summary.log; exit 1; }
  grep -E "^rank|pct" $O/potrf_q$q.log | cut -c1-300 | tee -a $O/summary.log
done
exit 0
