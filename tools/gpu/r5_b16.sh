#!/bin/bash
# r5 batch 16: DTR after removing the operand waterfall loops; is the segmented step order's intermittent wrong factor an L2 staleness? system-scope acquire A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b16
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {
  local name=$1; shift
  echo "== $name" | tee -a $O/summary.log
  env "$@" timeout -k 10 400 python tools/gpu/dtr_repeat.py 32768 16 > $O/$name.log 2>&1
  local rc=$?
  grep -E "FAILED|False" $O/$name.log | tail -4 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
echo "== perf column (after the waterfall fix)" | tee -a $O/summary.log
timeout -k 10 300 python tools/gpu/dtr_bench.py 16384 32768 65536 2>&1 | grep TIME | tee -a $O/summary.log
run step_w8_sysacq DPLASMA_DTR_LO_ORDER=step DPLASMA_DTR_STEPW=8 DPLASMA_DTR_SYSACQ=1 || exit 1
run step_w8 DPLASMA_DTR_LO_ORDER=step DPLASMA_DTR_STEPW=8 || exit 1
run step_w2 DPLASMA_DTR_LO_ORDER=step DPLASMA_DTR_STEPW=2 || exit 1
timeout -k 10 200 python -c "
import os, sys; os.environ['DPLASMA_DTR_LO_ORDER']='step'; os.environ['DPLASMA_DTR_STEPW']='8'; os.environ['DPLASMA_DTR_SYSACQ']='1'
sys.path.insert(0, 'tools/gpu'); import dtr_bench as b
for N in (16384, 32768, 65536): b.run(N, 'dtr')" 2>&1 | grep TIME | tee -a $O/summary.log
echo "== dtr_dist rehearsal 2 ranks" | tee -a $O/summary.log
DPLASMA_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 tools/gpu/dtr_dist_rehearsal.py 8192 1 2 > $O/rehearsal2.log 2>&1
echo "rc=$?" | tee -a $O/summary.log
grep -E "run |DTR-DIST|Error|error" $O/rehearsal2.log | head -12 | tee -a $O/summary.log
exit 0
