#!/bin/bash
# r5 batch 38: push-scheduled DTR -- bottom-level weight sweep at 16k / 32k (one workgroup per CU)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b38
mkdir -p $O
export PYTHONUNBUFFERED=1
perf() {
  echo "== $1" | tee -a $O/summary.log
  shift
  env "$@" timeout -k 10 200 python -c "
import sys; sys.path.insert(0, 'tools/gpu'); import dtr_bench as b
for N in (16384, 32768): b.run(N, 'dtr')" 2>&1 | grep TIME | tee -a $O/summary.log
}
perf default DPLASMA_DTR_SCHED=queue
perf panel_heavy DPLASMA_DTR_BL_W=75,65,400,800
perf trsm_heavy DPLASMA_DTR_BL_W=75,65,600,300
perf flat DPLASMA_DTR_BL_W=60,60,60,60
perf chain_light DPLASMA_DTR_BL_W=75,65,100,150
emu() {
  echo "== emul 2x4 64k $1" | tee -a $O/summary.log
  shift
  env DPLASMA_DTR_WG=256 "$@" timeout -k 10 300 python tools/emulate_potrf.py -N 65536 --grid 2x4 --bw 50 --lat 10 --reps 2 \
    2>&1 | grep EMUL | tee -a $O/summary.log
}
emu default DPLASMA_DTR_SCHED=queue
emu panel_heavy DPLASMA_DTR_BL_W=75,65,400,800
emu chain_light DPLASMA_DTR_BL_W=75,65,100,150
exit 0
