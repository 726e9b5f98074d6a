#!/bin/bash
# r4 batch 26: distributed LU panel rehearsal (2 ranks on one GPU, IPC exchange) -- per-column cost with the current
# kernel, without the wave priority, and with the kernel of commit 631c45e (before this session's changes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4b26
mkdir -p $O
export PYTHONUNBUFFERED=1
L=$(pwd)/dplasma_amd/lib
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|error|Error|us per column" $O/$name.log | grep -v amdgpu.ids | tail -4 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
R="python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1"
step cur 240 env DPLASMA_DIST_BACKEND=gloo $R --master-port 29541 tools/gpu/lu_dist_rehearsal.py 8192 512 || exit 1
step noprio 240 env DPLASMA_DIST_BACKEND=gloo DPLASMA_KERNELS_LIB=$L/libdplasma_kernels_noprio.so $R --master-port 29542 tools/gpu/lu_dist_rehearsal.py 8192 512 || exit 1
step old 240 env DPLASMA_DIST_BACKEND=gloo DPLASMA_KERNELS_LIB=$L/libdplasma_kernels_old.so $R --master-port 29543 tools/gpu/lu_dist_rehearsal.py 8192 512 || exit 1
exit 0
