#!/bin/bash
# r5 batch 47: bottom-level weights, heavier chain weightings around the adopted 400 / 800 (16k / 32k, 1 WG per CU)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b47
mkdir -p $O
export PYTHONUNBUFFERED=1
perf() {
  echo "== $1" | tee -a $O/summary.log
  shift
  env "$@" timeout -k 10 200 python -c "
import sys; sys.path.insert(0, 'tools/gpu'); import dtr_bench as b
for N in (16384, 32768): b.run(N, 'dtr')" 2>&1 | grep TIME | tee -a $O/summary.log
}
perf adopted DPLASMA_DTR_SCHED=queue
perf x2 DPLASMA_DTR_BL_W=75,65,800,1600
perf potrf_only DPLASMA_DTR_BL_W=75,65,175,1200
perf trsm400_potrf400 DPLASMA_DTR_BL_W=75,65,400,400
perf adopted_again DPLASMA_DTR_SCHED=queue
exit 0
