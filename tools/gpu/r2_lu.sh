#!/bin/bash
# LU look-ahead on one MI355X: LU GPU tests, then DGETRF 32k / 64k with and without look-ahead.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_lu.py tests/test_lu_qr.py -x -q -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/lu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/lu_tests.log; echo "lu tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
: > gpurun_out/lu_bench.log
for N in 32768 65536; do
  for LA in 0 1; do
    DPLASMA_LU_LOOKAHEAD=$LA timeout -k 10 240 python tools/bench_algo.py getrf_1d -N $N --nb 512 --runs 2 >> gpurun_out/lu_bench.log 2>&1
    rc=$?; echo "LA=$LA N=$N rc=$rc" >> gpurun_out/lu_bench.log; tail -2 gpurun_out/lu_bench.log
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
