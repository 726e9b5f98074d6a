#!/bin/bash
# r6 batch 7: LU replay 2x4 64k with exact panel slots + RNF (gather) and chunked exchanges; DTR probe v3 (snapshot)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b7
mkdir -p $O
export PYTHONUNBUFFERED=1
for cfg in "gather 1 2" "gather 0 2" "gather 1 1"; do
  set -- $cfg
  echo "== replay 2x4 64k panel=$1 RNF=$2 chunks=$3" | tee -a $O/summary.log
  DPLASMA_LU_PANEL=$1 DPLASMA_LU_RNF=$2 DPLASMA_LU_CHUNKS=$3 timeout -k 10 400 python tools/replay_lu.py -N 65536 --nb 512 \
    --grid 2x4 --xlat 3.3 --xgmi 2 > $O/rp_$1_$2_$3.log 2>&1 || { tail -30 $O/rp_$1_$2_$3.log | tee -a $O/summary.log; exit 1; }
  grep -E "^rank" $O/rp_$1_$2_$3.log | tr '\n' ' ' | tee -a $O/summary.log; echo | tee -a $O/summary.log
  grep -o '"pct_peak": [0-9.]*' $O/rp_$1_$2_$3.log | tee -a $O/summary.log
done
echo "== DTR probe v3 (POTRF input snapshot), queue, 512 WGs, 32k x 30" | tee -a $O/summary.log
DPLASMA_DTR_PROBE=1 DPLASMA_DTR_SNAP=1 DPLASMA_DTR_WG=512 timeout -k 10 500 python tools/gpu/dtr_repeat.py 32768 30 \
  > $O/probe.log 2>&1 || { tail -20 $O/probe.log | tee -a $O/summary.log; exit 1; }
grep -E "check=False|FAILED" $O/probe.log | sed -e 's/first (j, i, r, c, err): \[[^]]*\]//' | cut -c1-700 | tail -12 | tee -a $O/summary.log
exit 0
