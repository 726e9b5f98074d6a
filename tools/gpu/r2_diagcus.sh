#!/bin/bash
# DPOTRF with the diagonal-tile kernel on a CU-reserved stream (DPLASMA_DIAG_CUS=n) vs shared.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
: > gpurun_out/diagcus.log
for N in 16384 32768 65536; do
  for C in 0 4 8; do
    DPLASMA_DIAG_CUS=$C timeout -k 10 300 python bench.py -N $N --steps 3 --warmup 1 --no-check > gpurun_out/dc.log 2>&1
    rc=$?; echo "N=$N DIAG_CUS=$C $(grep -o '"value": [0-9.]*' gpurun_out/dc.log)" | tee -a gpurun_out/diagcus.log
    [ $rc -ne 0 ] && { tail -5 gpurun_out/dc.log; exit $rc; }
  done
done
exit 0
