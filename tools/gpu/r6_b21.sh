#!/bin/bash
# r6 batch 21: DTR push scheduler -- bottom-level priority resolution (DPLASMA_DTR_BUCKETS) and weights
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b21
mkdir -p $O
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
for cfg in "b22:" "b40:DPLASMA_DTR_BUCKETS=40" "b62:DPLASMA_DTR_BUCKETS=62" "b126:DPLASMA_DTR_BUCKETS=126" \
           "b62w:DPLASMA_DTR_BUCKETS=62 DPLASMA_DTR_BL_W=75,65,250,500" "b62w2:DPLASMA_DTR_BUCKETS=62 DPLASMA_DTR_BL_W=75,65,175,300"; do
  tag=${cfg%%:*}; e=${cfg#*:}
  echo "== $tag $e" | tee -a $O/summary.log
  env $e timeout -k 10 240 python tools/gpu/dtr_bench.py --engine dtr --reps 4 ${NS:-16384 32768} > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  grep TIME $O/$tag.log | cut -c1-150 | tee -a $O/summary.log
done
exit 0
