#!/bin/bash
# r4 batch 6: DTR per-task timeline + device-resident LU-QR (tests, 16k/32k timing)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r4b6
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_capi.py -k "native_gpu" -m gpu > gpurun_out/r4b6/capi_native.log 2>&1
rc=$?; tail -5 gpurun_out/r4b6/capi_native.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/gpu/dtr_trace_run.py 8192 gpurun_out/r4b6/dtr8k.npz > gpurun_out/r4b6/dtr8k.log 2>&1
rc=$?; cat gpurun_out/r4b6/dtr8k.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/gpu/dtr_trace_run.py 32768 gpurun_out/r4b6/dtr32k.npz > gpurun_out/r4b6/dtr32k.log 2>&1
rc=$?; cat gpurun_out/r4b6/dtr32k.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_lu_qr.py -m gpu > gpurun_out/r4b6/luqr_tests.log 2>&1
rc=$?; tail -8 gpurun_out/r4b6/luqr_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/gpu/luqr_prof.py 16384 512 > gpurun_out/r4b6/luqr16k.log 2>&1
rc=$?; grep "run " gpurun_out/r4b6/luqr16k.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/gpu/luqr_prof.py 32768 512 > gpurun_out/r4b6/luqr32k.log 2>&1
rc=$?; grep "run " gpurun_out/r4b6/luqr32k.log; exit $rc
