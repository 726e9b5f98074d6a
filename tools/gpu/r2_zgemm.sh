#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_zgemm_gpu.py tests/test_qr.py -x -q -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/zgemm_tests.log 2>&1
rc=$?; tail -4 gpurun_out/zgemm_tests.log; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/gpu/zgemm_bench.py 8192 16384 32768 > gpurun_out/zgemm_bench.log 2>&1
rc=$?; cat gpurun_out/zgemm_bench.log; exit $rc
