#!/bin/bash
# r6 batch 18: QR secondary metrics after the panel-kernel changes (flat 64k / 32k, HQR a=4 32k)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b18
mkdir -p $O
export PYTHONUNBUFFERED=1
run() { echo "== $*" | tee -a $O/summary.log; timeout -k 10 300 python tools/bench_algo.py "$@" > $O/last.log 2>&1 \
  || { tail -20 $O/last.log | tee -a $O/summary.log; return 1; }; grep TIME $O/last.log | tee -a $O/summary.log; }
run geqrf -N 65536 --nb 256 --runs 2 && run geqrf -N 32768 --nb 256 --runs 2 && \
run geqrf -N 32768 --nb 256 --tree hqr --qr-a 4 --runs 2
