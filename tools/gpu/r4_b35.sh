#!/bin/bash
# r4 batch 35: LU-QR 32k with the bulk updates capped (QR and LU REST as grid-stride GEMMs of n workgroups)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4b35
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "^run|Error|error" $O/$name.log | tail -4 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step base 200 python tools/gpu/luqr_syncdebug.py 32768 256 || exit 1
DPLASMA_QR_REST_CAP=224 DPLASMA_LU_REST_CAP=224 step cap224 200 python tools/gpu/luqr_syncdebug.py 32768 256 || exit 1
DPLASMA_QR_REST_CAP=480 DPLASMA_LU_REST_CAP=480 step cap480 200 python tools/gpu/luqr_syncdebug.py 32768 256 || exit 1
DPLASMA_QR_REST_CAP=240 step qrcap240 200 python tools/gpu/luqr_syncdebug.py 32768 256 || exit 1
exit 0
