#!/bin/bash
# CU-reserved diagonal stream (DPLASMA_DIAG_CUS) with the multi-workgroup tile kernel, 16k/32k/64k.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
out=gpurun_out/diagcus2.log; : > $out
for N in 16384 32768 65536; do
  for cus in 0 16 32; do
    for la in 1 2; do
      echo "N=$N DIAG_CUS=$cus LA=$la" >> $out
      DPLASMA_DIAG_CUS=$cus DPLASMA_POTRF_LOOKAHEAD=$la timeout -k 10 120 python bench.py -N $N --steps 2 --warmup 1 \
        --no-check 2>&1 | grep TIME >> $out || { cat $out; exit 1; }
    done
  done
done
cat $out
