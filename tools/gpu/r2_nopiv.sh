#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_lu.py -x -q -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/lu_gpu_tests.log 2>&1 || { tail -20 gpurun_out/lu_gpu_tests.log; exit 1; }
tail -1 gpurun_out/lu_gpu_tests.log
for N in 32768 65536; do
  timeout -k 10 300 python tools/bench_algo.py getrf_nopiv -N $N --nb 512 --runs 2 2>&1 | grep TIME || exit 1
done
