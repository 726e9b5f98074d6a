#!/bin/bash
# r6 batch 19: DGETRF one GPU -- look-ahead re-measured with the tagged panel kernel (r2's look-ahead numbers
# were taken with the grid-barrier panel), base block width 64 vs 32
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b19
mkdir -p $O
export PYTHONUNBUFFERED=1
for N in 32768 65536; do
  for cfg in "la0_bw64:DPLASMA_LU_LOOKAHEAD=0" "la1_bw64:DPLASMA_LU_LOOKAHEAD=1" "la1_bw32:DPLASMA_LU_LOOKAHEAD=1 DPLASMA_LU_BW=32"; do
    tag=${cfg%%:*}; e=${cfg#*:}
    echo "== $N $tag" | tee -a $O/summary.log
    env $e timeout -k 10 240 python tools/bench_algo.py getrf_1d -N $N --nb 512 --runs 2 > $O/${N}_$tag.log 2>&1 || exit 1
    grep TIME $O/${N}_$tag.log | cut -c1-140 | tee -a $O/summary.log
  done
done
exit 0
