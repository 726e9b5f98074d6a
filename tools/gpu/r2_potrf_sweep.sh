#!/bin/bash
# DPOTRF one-GPU sweep of the look-ahead depth and panel-TRSM kind at the per-GPU sizes of 1..8 GPUs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
out=gpurun_out/potrf_sweep.log
: > $out
for N in 16384 32768 65536; do
  for la in 1 2; do
    for tk in rb gemm; do
      st=3; [ $N -eq 65536 ] && st=2
      echo "N=$N LA=$la TRSM=$tk" >> $out
      DPLASMA_POTRF_LOOKAHEAD=$la DPLASMA_POTRF_TRSM=$tk timeout -k 10 120 python bench.py -N $N --steps $st --warmup 1 \
          --no-check 2>&1 | grep "TIME" >> $out || { echo "failed N=$N la=$la tk=$tk"; cat $out; exit 1; }
    done
  done
done
cat $out
