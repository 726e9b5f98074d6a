#!/bin/bash
# r5 batch 44: tagged LU block kernel with the record published before the rest of the rank-1 update
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b44
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|rror|TIME|us/column" $O/$name.log | grep -v amdgpu.ids | tail -8 | cut -c1-170 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step block 120 python tools/gpu/lu_block_bench.py 256 1024 8192 32768 65536 || exit 1
step lu_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lu.py tests/test_lu_qr.py -m gpu || exit 1
step getrf32k 200 python tools/bench_algo.py getrf_1d -N 32768 --nb 512 --runs 2 || exit 1
step getrf64k 300 python tools/bench_algo.py getrf_1d -N 65536 --nb 512 --runs 2 || exit 1
exit 0
