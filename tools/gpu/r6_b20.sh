#!/bin/bash
# r6 batch 20: DTR Cholesky -- narrower first panel blocks (DPLASMA_DTR_HEAD) and single-panel tail
# (DPLASMA_DTR_DEFER_MIN_TILES) at 16k / 32k
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b20
mkdir -p $O
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
for cfg in "base:" "h1:DPLASMA_DTR_HEAD=1" "h2:DPLASMA_DTR_HEAD=2" "h11:DPLASMA_DTR_HEAD=1,1" "h112:DPLASMA_DTR_HEAD=1,1,2" \
           "h12:DPLASMA_DTR_HEAD=1,2" "t8:DPLASMA_DTR_DEFER_MIN_TILES=8" "h1t8:DPLASMA_DTR_HEAD=1 DPLASMA_DTR_DEFER_MIN_TILES=8"; do
  tag=${cfg%%:*}; e=${cfg#*:}
  echo "== $tag $e" | tee -a $O/summary.log
  env $e timeout -k 10 240 python tools/gpu/dtr_bench.py --engine dtr --reps 4 ${NS:-16384 32768} > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  grep TIME $O/$tag.log | cut -c1-150 | tee -a $O/summary.log
done
exit 0
