#!/bin/bash
# r6 batch 36: end-to-end QR with the panel kernel's grid policy knobs (GMIN 8, RMAX 64) vs default, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b36
mkdir -p $O
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
run() { local tag=$1; shift; env $E timeout -k 10 300 python tools/bench_algo.py "$@" > $O/last.log 2>&1 \
  || { tail -20 $O/last.log; return 1; }; echo "$tag $* :: $(grep TIME $O/last.log | tail -1 | grep -o '[0-9.]* gflops')" | tee -a $O/summary.log; }
for r in 1 2; do
  for cfg in "def:" "g8r64:DPLASMA_QP_GMIN=8 DPLASMA_QP_RMAX=64"; do
    tag=${cfg%%:*}; E=${cfg#*:}
    run $tag geqrf -N 32768 --nb 256 --runs 2 || exit 1
    run $tag geqrf -N 32768 --nb 256 --tree hqr --qr-a 4 --runs 2 || exit 1
    run $tag geqrf -N 16384 --nb 256 --tree hqr --qr-a 4 --runs 2 || exit 1
  done
done
for cfg in "def:" "g8r64:DPLASMA_QP_GMIN=8 DPLASMA_QP_RMAX=64"; do
  tag=${cfg%%:*}; E=${cfg#*:}
  run $tag geqrf -N 65536 --nb 256 --runs 2 || exit 1
done
exit 0
