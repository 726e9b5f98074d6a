#!/bin/bash
# r6 batch 14: HQR 2x4 64k rank replay (config 4) with VSEND + full-duplex links; LU replay sensitivity (4 hw queues,
# 65 GB/s links)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b14
mkdir -p $O
export PYTHONUNBUFFERED=1
for v in 1 0; do
  echo "== HQR replay 2x4 64k NB=256 a=0 all ranks, VSEND=$v (bw 65, lat 10), 16 hw queues" | tee -a $O/summary.log
  DPLASMA_QR_VSEND=$v GPU_MAX_HW_QUEUES=16 timeout -k 10 700 python tools/replay_hqr.py -N 65536 --nb 256 --grid 2x4 --ranks all \
    --bw 65 --lat 10 > $O/hqr_v$v.log 2>&1 || { tail -20 $O/hqr_v$v.log | tee -a $O/summary.log; exit 1; }
  grep -E "^rank" $O/hqr_v$v.log | awk '{print $4}' | tr '\n' ' ' | tee -a $O/summary.log; echo | tee -a $O/summary.log
  grep -o '"pct_peak": [0-9.]*' $O/hqr_v$v.log | tee -a $O/summary.log
done
for cfg in "4 50" "16 65"; do
  set -- $cfg
  echo "== LU replay 2x4 64k gather, hw queues $1, bw $2" | tee -a $O/summary.log
  DPLASMA_LU_PANEL=gather timeout -k 10 400 python tools/replay_lu.py -N 65536 --nb 512 --grid 2x4 --hw-queues $1 --bw $2 \
    > $O/lu_q$1_bw$2.log 2>&1 || { tail -20 $O/lu_q$1_bw$2.log | tee -a $O/summary.log; exit 1; }
  grep -E "^rank" $O/lu_q$1_bw$2.log | awk '{print $4}' | tr '\n' ' ' | tee -a $O/summary.log; echo | tee -a $O/summary.log
  grep -o '"pct_peak": [0-9.]*' $O/lu_q$1_bw$2.log | tee -a $O/summary.log
done
exit 0
