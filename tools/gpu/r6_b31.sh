#!/bin/bash
# r6 batch 31: A/B on one box -- new one-process DGETRF defaults vs look-ahead off / 64-column blocks (both with the
# deferred left interchanges), alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b31
mkdir -p $O
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
for N in 32768 65536; do
  for cfg in "new:" "old:DPLASMA_LU_LOOKAHEAD=0 DPLASMA_LU_BW=64" "new2:" "old2:DPLASMA_LU_LOOKAHEAD=0 DPLASMA_LU_BW=64" "new3:" "old3:DPLASMA_LU_LOOKAHEAD=0 DPLASMA_LU_BW=64"; do
    tag=${cfg%%:*}; e=${cfg#*:}
    env $e timeout -k 10 240 python tools/bench_algo.py getrf_1d -N $N --nb 512 --runs 2 > $O/${N}_$tag.log 2>&1 || { tail -5 $O/${N}_$tag.log; exit 1; }
    echo "$N $tag $(grep TIME $O/${N}_$tag.log | tail -1 | grep -o '[0-9.]* gflops')" | tee -a $O/summary.log
  done
done
exit 0
