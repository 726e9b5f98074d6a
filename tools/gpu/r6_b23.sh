#!/bin/bash
# r6 batch 23: DTR push scheduler idle back-off cap (DPLASMA_DTR_NAP) x priority weights, 16k / 32k / 64k
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b23
mkdir -p $O
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
for cfg in "base:" "nap32:DPLASMA_DTR_NAP=32" "nap64:DPLASMA_DTR_NAP=64" "nap128:DPLASMA_DTR_NAP=128" \
           "nap64w:DPLASMA_DTR_NAP=64 DPLASMA_DTR_BUCKETS=62 DPLASMA_DTR_BL_W=75,65,250,500" \
           "w:DPLASMA_DTR_BUCKETS=62 DPLASMA_DTR_BL_W=75,65,250,500"; do
  tag=${cfg%%:*}; e=${cfg#*:}
  echo "== $tag $e" | tee -a $O/summary.log
  env $e timeout -k 10 300 python tools/gpu/dtr_bench.py --engine dtr --reps 4 ${NS:-16384 32768} > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  grep TIME $O/$tag.log | cut -c1-150 | tee -a $O/summary.log
done
DPLASMA_DTR_NAP=64 timeout -k 10 200 python -u tools/gpu/dtr_trace_run.py 16384 gpurun_out/dtr16k_nap.npz > gpurun_out/dtr16k_nap.log 2>&1 || exit 1
head -8 gpurun_out/dtr16k_nap.log; grep -A4 "^POTRF(1)" gpurun_out/dtr16k_nap.log
exit 0
