#!/bin/bash
# r5 batch 17: distributed DTR 2-process rehearsal with per-run residual / bad-tile report; the same grid emulated
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b17
mkdir -p $O
export PYTHONUNBUFFERED=1
echo "== emulation 1x2 8192 column" | tee -a $O/summary.log
timeout -k 10 200 python tools/emulate_potrf.py -N 8192 --grid 1x2 --order column --check --reps 3 > $O/emul12.log 2>&1 || exit 1
grep -E "resid|ms" $O/emul12.log | tail -4 | tee -a $O/summary.log
echo "== rehearsal 2 ranks 1x2 column" | tee -a $O/summary.log
DPLASMA_DTR_LO_ORDER=column DPLASMA_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 tools/gpu/dtr_dist_rehearsal.py 8192 1 4 > $O/rehearsal2.log 2>&1
echo "rc=$?" | tee -a $O/summary.log
grep -E "run |DTR-DIST|Error|error" $O/rehearsal2.log | head -12 | tee -a $O/summary.log
exit 0
