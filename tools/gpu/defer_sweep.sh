#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
: > gpurun_out/defer_sweep.log
for D in ${DS:-2 4 6 8}; do
  for MT in ${MTS:-24}; do
    DPLASMA_POTRF_DEFER=$D DPLASMA_POTRF_DEFER_MIN_TILES=$MT timeout -k 10 200 python bench.py --steps 2 --warmup 1 > gpurun_out/ds.log 2>&1
    rc=$?; echo "D=$D MIN=$MT $(grep -o '"value": [0-9.]*' gpurun_out/ds.log)" | tee -a gpurun_out/defer_sweep.log
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
