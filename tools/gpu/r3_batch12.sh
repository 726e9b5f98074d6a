#!/bin/bash
# C ABI GPU tests (one-process + multi-process native engine, F77 on BLACS grids of processes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_capi.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/b12_capi.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|FAIL" gpurun_out/b12_capi.log | tail -20; echo "capi rc=$rc"
exit $rc
