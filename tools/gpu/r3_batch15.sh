#!/bin/bash
# One-GPU DPOTRF at the per-rank share sizes: deferred-update depth x the tail threshold (plain look-ahead below it).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
OUT=gpurun_out/b15_potrf_defer.log
: > $OUT
for N in 16384 32768; do for D in 2 3 4 6; do for MT in 8 16 24 40; do
  v=$(DPLASMA_POTRF_DEFER=$D DPLASMA_POTRF_DEFER_MIN_TILES=$MT timeout -k 10 120 python bench.py -N $N --steps 6 --warmup 2 --no-check 2>/dev/null \
      | grep metric | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1000,2))") || { echo "N=$N D=$D MT=$MT failed"; exit 1; }
  echo "N=$N DEFER=$D MIN_TILES=$MT: $v TF/s" | tee -a $OUT
done; done; done
exit 0
