#!/bin/bash
# r6 batch 11: (1) DTR at two workgroups per CU with the compiler-visible M_k stores (the root-cause fix), stress probe;
# (2) kernel trace of LU replay rank 4 (gather, p2p, chunks 2, 16 hw queues); (3) HQR / POTRF replays, 4 vs 16 queues
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b11
mkdir -p $O
export PYTHONUNBUFFERED=1
echo "== DTR 512 WGs after the fix, probe + snapshot, 32k x 40" | tee -a $O/summary.log
DPLASMA_DTR_PROBE=1 DPLASMA_DTR_SNAP=1 DPLASMA_DTR_WG=512 timeout -k 10 600 python tools/gpu/dtr_repeat.py 32768 40 \
  > $O/probe.log 2>&1 || { tail -20 $O/probe.log | tee -a $O/summary.log; exit 1; }
grep -E "check=False|FAILED" $O/probe.log | sed -e 's/first (j, i, r, c, err): \[[^]]*\]//' -e 's/counters off.*//' | cut -c1-600 | tail -6 | tee -a $O/summary.log
echo "== DTR 512 WGs after the fix, plain (no probe), 16k x 40 and 32k x 20" | tee -a $O/summary.log
DPLASMA_DTR_WG=512 timeout -k 10 400 python tools/gpu/dtr_repeat.py 16384 40 > $O/p16.log 2>&1 || { tail -20 $O/p16.log | tee -a $O/summary.log; exit 1; }
grep -E "FAILED" $O/p16.log | tee -a $O/summary.log
DPLASMA_DTR_WG=512 timeout -k 10 400 python tools/gpu/dtr_repeat.py 32768 20 > $O/p32.log 2>&1 || { tail -20 $O/p32.log | tee -a $O/summary.log; exit 1; }
grep -E "FAILED" $O/p32.log | tee -a $O/summary.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
echo "== trace LU replay rank 4" | tee -a $O/summary.log
DPLASMA_LU_PANEL=gather DPLASMA_LU_RNF=0 timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o rank4 -- \
  python tools/replay_lu.py -N 65536 --nb 512 --grid 2x4 --ranks 4 --xlat 3.3 --xgmi 2 --hw-queues 16 > $O/rp.log 2>&1 \
  || { tail -30 $O/rp.log | tee -a $O/summary.log; exit 1; }
grep -E "^rank" $O/rp.log | tee -a $O/summary.log
bash tools/gpu/r6_b10.sh > $O/b10.log 2>&1 || { tail -20 $O/b10.log | tee -a $O/summary.log; exit 1; }
cat gpurun_out/r6b10/summary.log >> $O/summary.log
exit 0
