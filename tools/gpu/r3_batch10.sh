#!/bin/bash
# Multi-process native C ABI (ranks sharing the GPU, file transport) + the one-process C tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_capi.py -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/b10_capi.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed|max rel|Error|error" gpurun_out/b10_capi.log | tail -40; echo "capi rc=$rc"
exit $rc
