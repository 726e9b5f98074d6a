#!/bin/bash
# Session checks: DTD QR / incpiv LU (batched kinds) and the native C ABI additions on the GPU, the
# DTD testing programs at 4k, then a kernel-trace profile of DGEQRF 32k.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_dtd_factor.py tests/test_dtd.py tests/test_capi.py -m gpu -x -v \
    --timeout 120 --timeout-method thread > gpurun_out/gpu_s5.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_s5.log; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/cli_dtd.log
for a in "dgeqrf_dtd -N 4096 -t 256 -i 32 -x" "dgeqrf -N 4096 -t 256 -i 32 -x" \
         "dgetrf_incpiv_dtd -N 4096 -t 256 -i 32 -x" "dgetrf_incpiv -N 4096 -t 256 -i 32 -x"; do
  (cd /tmp && PYTHONPATH=$R timeout -k 10 200 python -m dplasma_amd.testing $a >> $R/gpurun_out/cli_dtd.log 2>&1)
  rc=$?; [ $rc -ne 0 ] && { tail -20 gpurun_out/cli_dtd.log; exit $rc; }
done
grep -E "TIME|CORRECT|SUSP" gpurun_out/cli_dtd.log
QR_N=32768 bash tools/gpu/prof_qr.sh
