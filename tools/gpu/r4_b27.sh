#!/bin/bash
# r4 batch 27: LU-QR (32-column LU panel blocks by default now) and HQR with the bulk (REST) updates capped to
# n workgroups so the next step's panels find CUs beside them.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4b27
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|error|Error|TF/s|TIME" $O/$name.log | grep -v amdgpu.ids | tail -4 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step luqr_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lu_qr.py -m gpu || exit 1
step luqr32k 300 python tools/gpu/luqr_syncdebug.py 32768 256 || exit 1
for c in 448 384 320; do
  step luqr32k_cap$c 300 env DPLASMA_QR_REST_CAP=$c DPLASMA_LU_REST_CAP=$c python tools/gpu/luqr_syncdebug.py 32768 256 || exit 1
done
step hqr32k_a4 200 python tools/bench_algo.py geqrf -N 32768 --nb 256 --ib 32 --runs 2 --tree hqr --qr-llvl 1 --qr-hlvl 0 --qr-a 4 || exit 1
step hqr32k_a4_cap384 200 env DPLASMA_QR_REST_CAP=384 python tools/bench_algo.py geqrf -N 32768 --nb 256 --ib 32 --runs 2 --tree hqr --qr-llvl 1 --qr-hlvl 0 --qr-a 4 || exit 1
exit 0
