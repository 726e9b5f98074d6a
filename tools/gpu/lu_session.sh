#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "lu or getrf or piv or gesv" --timeout 120 --timeout-method thread > gpurun_out/lu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/lu_tests.log; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/algo.log
for N in ${LU_NS:-16384 32768}; do
  timeout -k 10 300 python tools/bench_algo.py getrf_1d -N $N --nb 512 --runs 2 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/algo.log
  rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && exit $rc
done
exit 0
