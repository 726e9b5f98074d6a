#!/bin/bash
# POTRF with the bulk trailing updates as capped grid-stride GEMM launches (DPLASMA_POTRF_RESERVE CUs
# kept free for the panel chain): correctness first (GPU potrf tests with a reserve), then a sweep.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
out=gpurun_out/reserve.log
: > $out
DPLASMA_POTRF_RESERVE=16 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 \
    --timeout-method thread -k "potrf or gemm" >> $out 2>&1 || { tail -30 $out; exit 1; }
tail -2 $out
for N in 16384 32768 65536; do
  for R in ${RESERVES:-0 8 16 32}; do
    st=5; [ $N -eq 65536 ] && st=2
    echo "N=$N RESERVE=$R" >> $out
    DPLASMA_POTRF_RESERVE=$R timeout -k 10 240 python bench.py -N $N --steps $st --warmup 1 --no-check \
        >> $out 2>&1 || { tail -20 $out; exit 1; }
  done
done
grep -E "^N=|TIME" $out
