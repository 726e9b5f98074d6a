#!/bin/bash
# CU-reserved critical stream (tile POTRF + panel TRSM) vs shared streams, with defer depth and look-ahead.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
out=gpurun_out/diagcus3.log; : > $out
run() {
  echo "$*" >> $out
  env "$@" timeout -k 10 120 python bench.py -N $N --steps 2 --warmup 1 --no-check 2>&1 | grep TIME >> $out || { cat $out; exit 1; }
}
for N in 16384 32768; do
  run N=$N DPLASMA_DIAG_CUS=0
  for cus in 16 32 64; do
    for d in 4 2; do
      for la in 1 2; do
        run N=$N DPLASMA_DIAG_CUS=$cus DPLASMA_POTRF_DEFER=$d DPLASMA_POTRF_LOOKAHEAD=$la
      done
    done
  done
done
N=65536
run N=$N DPLASMA_DIAG_CUS=0
run N=$N DPLASMA_DIAG_CUS=32 DPLASMA_POTRF_LOOKAHEAD=2
run N=$N DPLASMA_DIAG_CUS=16 DPLASMA_POTRF_LOOKAHEAD=2
cat $out
