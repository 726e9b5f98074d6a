#!/bin/bash
# r6 batch 37: panel kernel with at least 8 workgroups (DPLASMA_QP_GMIN=8; TT kills 2 -> 8): HQR config 4 rank replay,
# then one-GPU flat 32k / HQR a=4 32k A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b37
mkdir -p $O
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
( while true; do date >> $O/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
echo "== HQR replay 2x4 64k GMIN=8" | tee -a $O/summary.log
DPLASMA_QP_GMIN=8 GPU_MAX_HW_QUEUES=16 timeout -k 10 900 python tools/replay_hqr.py -N 65536 --nb 256 --grid 2x4 --bw 65 --lat 10 \
  > $O/rp.log 2>&1 || { tail -30 $O/rp.log | tee -a $O/summary.log; exit 1; }
grep -E "^rank|pct_peak" $O/rp.log | tee -a $O/summary.log
run() { local tag=$1; shift; env $E timeout -k 10 300 python tools/bench_algo.py "$@" > $O/last.log 2>&1 \
  || { tail -20 $O/last.log; return 1; }; echo "$tag $* :: $(grep TIME $O/last.log | tail -1 | grep -o '[0-9.]* gflops')" | tee -a $O/summary.log; }
for cfg in "def:" "g8:DPLASMA_QP_GMIN=8" "def2:" "g8b:DPLASMA_QP_GMIN=8"; do
  tag=${cfg%%:*}; E=${cfg#*:}
  run $tag geqrf -N 32768 --nb 256 --runs 2 || exit 1
  run $tag geqrf -N 32768 --nb 256 --tree hqr --qr-a 4 --runs 2 || exit 1
done
exit 0
