#!/bin/bash
# r5 batch 18: distributed DTR rehearsals -- 2, 4 and 8 processes sharing one GPU (each its share of the workgroups)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b18
mkdir -p $O
export PYTHONUNBUFFERED=1
reh() {   # name nproc P N order
  echo "== $1: $2 processes P=$3 N=$4 order=$5" | tee -a $O/summary.log
  DPLASMA_DTR_LO_ORDER=$5 DPLASMA_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nproc-per-node $2 \
    --master-addr 127.0.0.1 --master-port 29517 tools/gpu/dtr_dist_rehearsal.py $4 $3 3 > $O/$1.log 2>&1
  local rc=$?
  grep -E "run |DTR-DIST|Error|error" $O/$1.log | head -8 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
reh g12_16k 2 1 16384 column || exit 1
reh g22_16k 4 2 16384 column || exit 1
reh g24_16k 8 2 16384 column || exit 1
reh g24_16k_step 8 2 16384 step || exit 1
reh g24_32k 8 2 32768 column || exit 1
exit 0
