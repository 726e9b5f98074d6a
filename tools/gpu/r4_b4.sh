#!/bin/bash
# r4 batch 4: device task runtime Cholesky (small sizes first, bounded) + RCCL loopback rehearsals
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r4b4
export PYTHONUNBUFFERED=1
timeout -k 10 180 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_potrf_dtr.py -m gpu \
  > gpurun_out/r4b4/dtr_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r4b4/dtr_tests.log; echo "dtr tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/gpu/dtr_bench.py 8192 16384 32768 > gpurun_out/r4b4/dtr_bench.log 2>&1
rc=$?; cat gpurun_out/r4b4/dtr_bench.log; echo "dtr bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_loopback.py \
  "tests/test_capi.py::test_capi_native_dist_loopback_rccl" -m gpu > gpurun_out/r4b4/loopback.log 2>&1
rc=$?; tail -30 gpurun_out/r4b4/loopback.log; echo "loopback rc=$rc"; exit $rc
