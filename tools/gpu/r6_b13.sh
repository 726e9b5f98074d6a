#!/bin/bash
# r6 batch 13: LU 2x4 64k rank replay after LSEND split + full-duplex link accounting (16 hw queues)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b13
mkdir -p $O
export PYTHONUNBUFFERED=1
for cfg in "gather 0 2" "gather 0 4" "gather 1 2"; do
  set -- $cfg
  tag=$1_$2_$3
  echo "== replay 2x4 64k panel=$1 RNF=$2 chunks=$3 (bw 50, lat 15, xlat 3.3 + xgmi 2)" | tee -a $O/summary.log
  DPLASMA_LU_PANEL=$1 DPLASMA_LU_RNF=$2 DPLASMA_LU_CHUNKS=$3 timeout -k 10 400 python tools/replay_lu.py -N 65536 --nb 512 \
    --grid 2x4 --xlat 3.3 --xgmi 2 --hw-queues 16 > $O/rp_$tag.log 2>&1 || { tail -30 $O/rp_$tag.log | tee -a $O/summary.log; exit 1; }
  grep -E "^rank" $O/rp_$tag.log | awk '{print $4}' | tr '\n' ' ' | tee -a $O/summary.log; echo | tee -a $O/summary.log
  grep -o '"pct_peak": [0-9.]*' $O/rp_$tag.log | tee -a $O/summary.log
done
exit 0
