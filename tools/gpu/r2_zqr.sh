#!/bin/bash
# Complex stacked-domain QR engine (qr_panel_z.hip): GPU QR tests, then zgeqrf / cgeqrf rates
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_qr.py -x -v -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/zqr_tests.log 2>&1 || { grep -E "PASSED|FAILED|Error|error" gpurun_out/zqr_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/zqr_tests.log
for a in "z 8192" "z 16384" "z 32768" "c 16384"; do
  set -- $a
  timeout -k 10 300 python tools/bench_algo.py geqrf -N $2 --nb 256 --ib 32 --prec $1 --runs 2 2>&1 | grep TIME || exit 1
done
