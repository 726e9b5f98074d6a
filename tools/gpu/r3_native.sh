#!/bin/bash
# Native C ABI GPU tests (tests/capi/test_native.c via tests/test_capi.py) and the F77 layer.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_capi.py -m gpu -x -v --timeout 300 --timeout-method thread -s \
    > gpurun_out/native_capi.log 2>&1
rc=$?; grep -E "error|residual|FAIL|passed|failed|native C ABI" gpurun_out/native_capi.log | tail -40; exit $rc
