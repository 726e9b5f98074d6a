#!/bin/bash
# r6 batch 29: DGETRF one GPU with deferred left interchanges (default now) x panel block width x look-ahead
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b29
mkdir -p $O
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
for N in 32768 65536; do
  for cfg in "d:" "bw32:DPLASMA_LU_BW=32" "la1:DPLASMA_LU_LOOKAHEAD=1" "la1bw32:DPLASMA_LU_LOOKAHEAD=1 DPLASMA_LU_BW=32" "d2:" "bw32b:DPLASMA_LU_BW=32"; do
    tag=${cfg%%:*}; e=${cfg#*:}
    echo "== N=$N $tag $e" | tee -a $O/summary.log
    env $e timeout -k 10 240 python tools/bench_algo.py getrf_1d -N $N --nb 512 --runs 2 > $O/${N}_$tag.log 2>&1 || { tail -5 $O/${N}_$tag.log; exit 1; }
    grep TIME $O/${N}_$tag.log | tail -1 | cut -c1-140 | tee -a $O/summary.log
  done
done
exit 0
