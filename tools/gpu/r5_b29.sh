#!/bin/bash
# r5 batch 29: one workgroup per CU -- DTR list orders (column / step + segments) at 16k / 32k / 64k
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b29
mkdir -p $O
export PYTHONUNBUFFERED=1
perf() {
  echo "== $1" | tee -a $O/summary.log
  shift
  env "$@" timeout -k 10 240 python -c "
import sys; sys.path.insert(0, 'tools/gpu'); import dtr_bench as b
for N in (16384, 32768, 65536): b.run(N, 'dtr')" 2>&1 | grep TIME | tee -a $O/summary.log
}
perf column DPLASMA_DTR_LO_ORDER=column
perf step_w8 DPLASMA_DTR_LO_ORDER=step DPLASMA_DTR_STEPW=8
perf step_w2 DPLASMA_DTR_LO_ORDER=step DPLASMA_DTR_STEPW=2
perf step_w4 DPLASMA_DTR_LO_ORDER=step DPLASMA_DTR_STEPW=4
perf panel DPLASMA_DTR_LO_ORDER=panel
exit 0
