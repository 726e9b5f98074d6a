#!/bin/bash
# r4 batch 7: capped grid-stride GEMM without spills -> re-sweep CU reservation for DPOTRF and the
# LU look-ahead with a capped REST update.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r4b7
export PYTHONUNBUFFERED=1
L=gpurun_out/r4b7/sweep.log
: > $L
run() {  # label, env..., -- args
  local label=$1; shift
  echo "== $label" | tee -a $L
  env "$@" 2>&1 | grep -E "TIME|Error|error" | tee -a $L
  return ${PIPESTATUS[0]}
}
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_zgemm_gpu.py -m gpu -k "gemm" > gpurun_out/r4b7/gemm_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4b7/gemm_tests.log; [ $rc -ne 0 ] && exit $rc
for N in 32768 65536; do
  for R in 0 8 16 32; do
    run "potrf N=$N reserve=$R" DPLASMA_POTRF_RESERVE=$R timeout -k 10 200 python tools/bench_algo.py potrf -N $N --nb 512 --runs 2 || exit 1
  done
done
for N in 32768 65536; do
  run "getrf N=$N baseline" timeout -k 10 200 python tools/bench_algo.py getrf_1d -N $N --nb 512 --runs 2 || exit 1
  for C in 0 480 448 384; do
    run "getrf N=$N lookahead cap=$C" DPLASMA_LU_LOOKAHEAD=1 DPLASMA_LU_REST_CAP=$C timeout -k 10 200 python tools/bench_algo.py getrf_1d -N $N --nb 512 --runs 2 || exit 1
  done
done
exit 0
