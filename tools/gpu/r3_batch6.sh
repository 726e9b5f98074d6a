#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_lu_qr.py -m gpu -x -q --timeout 180 --timeout-method thread \
    > gpurun_out/b6_tests.log 2>&1
rc=$?; tail -2 gpurun_out/b6_tests.log; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
for N in 16384 32768; do
  timeout -k 10 300 python -m dplasma_amd.testing dgetrf_qrf -N $N -t 256 -x > gpurun_out/b6_luqr_$N.log 2>&1
  rc=$?; grep -E "TIME|SUCC|FAIL|Error|rror" gpurun_out/b6_luqr_$N.log | head -5; echo "getrf_qrf $N rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
