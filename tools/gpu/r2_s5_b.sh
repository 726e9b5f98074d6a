#!/bin/bash
# Follow-up: incremental-pivoting LU residual at 4k with and without DTD (the check result is printed,
# a SUSPICIOUS line is not a failure of this script), then the DGEQRF 32k kernel profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
mkdir -p gpurun_out
: > gpurun_out/cli_incpiv.log
for a in "dgetrf_incpiv -N 4096 -t 256 -i 32 -x" "dgetrf_incpiv_dtd -N 4096 -t 256 -i 32 -x" \
         "dgetrf_incpiv -N 4096 -t 256 -i 16 -x" "dgetrf_1d -N 4096 -t 256 -x"; do
  (cd /tmp && PYTHONPATH=$R timeout -k 10 200 python -m dplasma_amd.testing $a >> $R/gpurun_out/cli_incpiv.log 2>&1)
  rc=$?; [ $rc -gt 1 ] && { tail -20 gpurun_out/cli_incpiv.log; exit $rc; }
done
grep -E "TIME|CORRECT|SUSP" gpurun_out/cli_incpiv.log
QR_N=32768 bash tools/gpu/prof_qr.sh
