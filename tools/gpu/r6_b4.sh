#!/bin/bash
# r6 batch 4: LU rank replay 2x4 (p2p interchanges, look-ahead; gather vs dist panel with the measured hand-off),
# the w4 anomaly probe with the stream engine in between, DTR strip-hazard probe at 512 workgroups
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b4
mkdir -p $O
export PYTHONUNBUFFERED=1
echo "== replay plumbing 8k" | tee -a $O/summary.log
timeout -k 10 200 python tools/replay_lu.py -N 8192 --nb 512 --grid 2x4 --ranks 0,5 --xlat 3.3 --xgmi 2 > $O/rp8k.log 2>&1 \
  || { tail -30 $O/rp8k.log | tee -a $O/summary.log; exit 1; }
tail -1 $O/rp8k.log | cut -c1-300 | tee -a $O/summary.log
for mode in gather dist; do
  echo "== replay 2x4 64k panel=$mode" | tee -a $O/summary.log
  DPLASMA_LU_PANEL=$mode timeout -k 10 400 python tools/replay_lu.py -N 65536 --nb 512 --grid 2x4 --xlat 3.3 --xgmi 2 \
    > $O/rp64k_$mode.log 2>&1 || { tail -30 $O/rp64k_$mode.log | tee -a $O/summary.log; exit 1; }
  grep -E "^rank|pct_peak" $O/rp64k_$mode.log | cut -c1-400 | tee -a $O/summary.log
done
echo "== w4 queue probe with the stream engine" | tee -a $O/summary.log
env DPLASMA_DIST_BACKEND=gloo DPLASMA_DTR_WG=64 timeout -k 10 240 python -m torch.distributed.run \
  --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29704 tools/gpu/dtr_w4_queues.py 16384 \
  > $O/w4.log 2>&1 || { tail -20 $O/w4.log | tee -a $O/summary.log; exit 1; }
grep "N=" $O/w4.log | tee -a $O/summary.log
echo "== DTR strip-hazard probe, 512 workgroups, step order w2 + POTRF hold (the r5 stress), 32k x 30" | tee -a $O/summary.log
DPLASMA_DTR_PROBE=1 DPLASMA_DTR_WG=512 DPLASMA_DTR_LO_ORDER=step DPLASMA_DTR_STEPW=2 DPLASMA_DTR_HOLD=2550,0 \
  timeout -k 10 400 python tools/gpu/dtr_repeat.py 32768 30 > $O/probe.log 2>&1 || { tail -20 $O/probe.log | tee -a $O/summary.log; exit 1; }
grep -E "check=False|probe:|FAILED" $O/probe.log | cut -c1-600 | tail -12 | tee -a $O/summary.log
exit 0
