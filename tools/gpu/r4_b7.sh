#!/bin/bash
# r4 batch 7: DTR with a ticketed high list (tests, trace, bench); device-resident LU-QR at NB=256 under
# sync-debug; capped GEMM without spills (GEMM tests, POTRF reserve and LU look-ahead cap sweeps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4b7
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|error|Error|TF/s|TIME|span=|occupancy|rank |worst|run [0-9]" $O/$name.log | grep -v amdgpu.ids | tail -12 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step dtr_tests 240 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_potrf_dtr.py -m gpu || exit 1
step dtr_trace32k 200 python tools/gpu/dtr_trace_run.py 32768 $O/dtr32k.npz || exit 1
step dtr_bench 600 python tools/gpu/dtr_bench.py 16384 32768 65536 || exit 1
step luqr_sync8k 300 python tools/gpu/luqr_syncdebug.py 8192 256 || exit 1
step luqr_sync32k 600 python tools/gpu/luqr_syncdebug.py 32768 256 || exit 1
step luqr_cli8k 300 python -m dplasma_amd.testing dgetrf_qrf -N 8192 -t 256 -T 256 -x || exit 1
step gemm_tests 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "gemm" || exit 1
for N in 32768 65536; do
  for R in 0 16 32; do
    step potrf_${N}_res$R 200 env DPLASMA_POTRF_RESERVE=$R python tools/bench_algo.py potrf -N $N --nb 512 --runs 2 || exit 1
  done
  for C in 0 448 384; do
    step getrf_${N}_la_cap$C 200 env DPLASMA_LU_LOOKAHEAD=1 DPLASMA_LU_REST_CAP=$C python tools/bench_algo.py getrf_1d -N $N --nb 512 --runs 2 || exit 1
  done
done
exit 0
