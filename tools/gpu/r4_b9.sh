#!/bin/bash
# r4 batch 9: DTR low-list order (column blocks vs panel blocks) and deferral depth; capped GEMM
# (spill-free) re-sweep: DPOTRF CU reserve (stream engine), DGETRF look-ahead with a capped REST.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4b9
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|error|Error|TF/s|TIME|span=|occupancy" $O/$name.log | grep -v amdgpu.ids | tail -8 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step dtr_tests 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_potrf_dtr.py -m gpu || exit 1
step dtr_col_D4 500 env DPLASMA_DTR_LO_ORDER=column python tools/gpu/dtr_bench.py 16384 32768 65536 || exit 1
step dtr_col_D2 400 env DPLASMA_DTR_LO_ORDER=column DPLASMA_DTR_DEFER=2 python tools/gpu/dtr_bench.py 16384 32768 || exit 1
step dtr_trace32k_col 200 env DPLASMA_DTR_LO_ORDER=column python tools/gpu/dtr_trace_run.py 32768 $O/dtr32k_col.npz || exit 1
for N in 32768 65536; do
  for R in 16 32; do
    step potrf_${N}_res$R 200 env DPLASMA_POTRF_RESERVE=$R python -m dplasma_amd.testing dpotrf -N $N -t 512 -T 512 --nruns 2 || exit 1
  done
  step getrf_${N}_base 200 python tools/bench_algo.py getrf_1d -N $N --nb 512 --runs 2 || exit 1
  for C in 448 384; do
    step getrf_${N}_la_cap$C 200 env DPLASMA_LU_LOOKAHEAD=1 DPLASMA_LU_REST_CAP=$C python tools/bench_algo.py getrf_1d -N $N --nb 512 --runs 2 || exit 1
  done
done
exit 0
