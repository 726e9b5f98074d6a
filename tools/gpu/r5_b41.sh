#!/bin/bash
# r5 batch 41: distributed LU panel with the tagged local exchange -- IPC tests, LU suites, 2-process rehearsal
# (new kernels vs libdplasma_kernels_oldlu.so = the same tree with the previous grid-barrier dist panel)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=gpurun_out/r5b41
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|rror|TF/s|TIME|per column|pivots|ms" $O/$name.log | grep -v amdgpu.ids | tail -10 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
TR="python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1"
step lu_tests 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_lu_dist.py tests/test_lu.py tests/test_lu_qr.py -m gpu || exit 1
step reh_new 240 env DPLASMA_DIST_BACKEND=gloo $TR --master-port 29561 tools/gpu/lu_dist_rehearsal.py 8192 512 || exit 1
step reh_old 240 env DPLASMA_DIST_BACKEND=gloo DPLASMA_KERNELS_LIB=$R/dplasma_amd/lib/libdplasma_kernels_oldlu.so $TR --master-port 29562 tools/gpu/lu_dist_rehearsal.py 8192 512 || exit 1
step reh_new16k 300 env DPLASMA_DIST_BACKEND=gloo $TR --master-port 29563 tools/gpu/lu_dist_rehearsal.py 16384 512 || exit 1
exit 0
