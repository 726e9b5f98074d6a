#!/bin/bash
# r5 batch 30: LU-QR device-decided steps (predicated branches) vs the host-decided path; LU-QR GPU tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b30
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_lu_qr.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo "rc=$?" | tee -a $O/summary.log
grep -E "PASS|FAIL|Error|lu_tab|passed|failed" $O/tests.log | tail -30 | tee -a $O/summary.log
exit 0
