#!/bin/bash
# r6 batch 9: LU replay 2x4 64k with one hardware queue per stream (GPU_MAX_HW_QUEUES=16) vs HIP's default 4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b9
mkdir -p $O
export PYTHONUNBUFFERED=1
for cfg in "gather 0 2 16" "gather 1 2 16" "dist 0 2 16" "gather 0 2 4"; do
  set -- $cfg
  tag=$1_$2_$3_q$4
  echo "== replay 2x4 64k panel=$1 RNF=$2 chunks=$3 hw-queues=$4" | tee -a $O/summary.log
  DPLASMA_LU_PANEL=$1 DPLASMA_LU_RNF=$2 DPLASMA_LU_CHUNKS=$3 timeout -k 10 400 python tools/replay_lu.py -N 65536 --nb 512 \
    --grid 2x4 --xlat 3.3 --xgmi 2 --hw-queues $4 > $O/rp_$tag.log 2>&1 || { tail -30 $O/rp_$tag.log | tee -a $O/summary.log; exit 1; }
  grep -E "^rank" $O/rp_$tag.log | awk '{print $3}' | tr '\n' ' ' | tee -a $O/summary.log; echo | tee -a $O/summary.log
  grep -o '"pct_peak": [0-9.]*' $O/rp_$tag.log | tee -a $O/summary.log
done
echo "== DTR probe v5 (post mortem of published blocks), queue, 512 WGs, 32k x 40" | tee -a $O/summary.log
DPLASMA_DTR_PROBE=1 DPLASMA_DTR_SNAP=1 DPLASMA_DTR_WG=512 timeout -k 10 600 python tools/gpu/dtr_repeat.py 32768 40 \
  > $O/probe.log 2>&1 || { tail -20 $O/probe.log | tee -a $O/summary.log; exit 1; }
grep -E "check=False|FAILED" $O/probe.log | sed -e 's/first (j, i, r, c, err): \[[^]]*\]//' -e 's/counters off.*//' | cut -c1-1500 | tail -12 | tee -a $O/summary.log
exit 0
