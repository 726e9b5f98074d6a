#!/bin/bash
# CU-masked diagonal stream with ONLY the tile POTRF on it (DPLASMA_POTRF_DIAG_TRSM=0: the panel TRSM
# stays on the unmasked high-priority panel stream) -- the variant the earlier DIAG_CUS sweeps missed.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
out=gpurun_out/diag_notrsm.log
: > $out
for N in 16384 32768; do
  for D in 0 8 16 32; do
    echo "N=$N DIAG_CUS=$D DIAG_TRSM=0" >> $out
    DPLASMA_DIAG_CUS=$D DPLASMA_POTRF_DIAG_TRSM=0 timeout -k 10 200 python bench.py -N $N --steps 5 --warmup 1 \
        --no-check >> $out 2>&1 || { tail -20 $out; exit 1; }
  done
done
grep -E "^N=|TIME" $out
