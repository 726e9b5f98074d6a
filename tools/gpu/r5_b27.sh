#!/bin/bash
# r5 batch 27: HQR 2x4 replay (one TS domain per row, and a = 4 greedy: row-merged TT stacks); GPU QR/DTR tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b27
mkdir -p $O
export PYTHONUNBUFFERED=1
echo "== gpu tests qr + dtr" | tee -a $O/summary.log
timeout -k 10 600 python -u -m pytest tests/test_qr.py tests/test_potrf_dtr.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "rc=$?" | tee -a $O/summary.log
tail -3 $O/tests.log | tee -a $O/summary.log
echo "== replay hqr 2x4 64k a=0 (baseline config)" | tee -a $O/summary.log
timeout -k 10 500 python tools/replay_hqr.py -N 65536 --nb 256 --grid 2x4 --ranks 0,4 --bw 65 --lat 10 > $O/replay_a0.log 2>&1
echo "rc=$?" | tee -a $O/summary.log
tail -4 $O/replay_a0.log | tee -a $O/summary.log
echo "== replay hqr 2x4 64k greedy a=4 (row-merged)" | tee -a $O/summary.log
timeout -k 10 500 python tools/replay_hqr.py -N 65536 --nb 256 --grid 2x4 --ranks 0,4 --bw 65 --lat 10 --a 4 > $O/replay_a4.log 2>&1
echo "rc=$?" | tee -a $O/summary.log
tail -4 $O/replay_a4.log | tee -a $O/summary.log
echo "== replay hqr 2x4 64k greedy a=4 (pairwise TT)" | tee -a $O/summary.log
DPLASMA_QR_MERGE_TT=1 timeout -k 10 500 python tools/replay_hqr.py -N 65536 --nb 256 --grid 2x4 --ranks 0,4 --bw 65 --lat 10 --a 4 > $O/replay_a4_pair.log 2>&1
echo "rc=$?" | tee -a $O/summary.log
tail -4 $O/replay_a4_pair.log | tee -a $O/summary.log
exit 0
