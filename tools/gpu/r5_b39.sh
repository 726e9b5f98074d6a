#!/bin/bash
# r5 batch 39: LU block kernel pivot exchange -- tagged granules (default) vs flat counter vs XCD-sharded counter
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b39
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|rror|TF/s|TIME|us/column" $O/$name.log | grep -v amdgpu.ids | tail -8 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step lu_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lu.py -m gpu || exit 1
step block_tag 120 python tools/gpu/lu_block_bench.py 1024 8192 32768 65536 || exit 1
DPLASMA_LU_BLOCK=xcd step block_xcd 120 python tools/gpu/lu_block_bench.py 1024 8192 32768 65536 || exit 1
DPLASMA_LU_BLOCK=flat step block_flat 120 python tools/gpu/lu_block_bench.py 1024 8192 32768 65536 || exit 1
step getrf32k_tag 200 python tools/bench_algo.py getrf_1d -N 32768 --nb 512 --runs 2 || exit 1
DPLASMA_LU_BLOCK=flat step getrf32k_flat 200 python tools/bench_algo.py getrf_1d -N 32768 --nb 512 --runs 2 || exit 1
step getrf64k_tag 300 python tools/bench_algo.py getrf_1d -N 65536 --nb 512 --runs 2 || exit 1
DPLASMA_LU_BLOCK=flat step getrf64k_flat 300 python tools/bench_algo.py getrf_1d -N 65536 --nb 512 --runs 2 || exit 1
exit 0
