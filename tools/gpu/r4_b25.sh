#!/bin/bash
# r4 batch 25: panel kernels at wave priority 3 (VALU issue over co-resident GEMM waves); distributed LU panel
# with single-barrier argmax (IPC rehearsal test); getrf / LU-QR with and without the 32-column block + look-ahead.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4b25
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E "passed|failed|error|Error|TF/s|TIME|us/column|per column" $O/$name.log | grep -v amdgpu.ids | tail -8 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
step lu_tests 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_lu.py tests/test_gpu_lu_dist.py tests/test_lu_qr.py tests/test_qr.py -m gpu || exit 1
step getrf32k 200 python tools/bench_algo.py getrf_1d -N 32768 --nb 512 --runs 2 || exit 1
step getrf32k_la_bw32 200 env DPLASMA_LU_BW=32 DPLASMA_LU_LOOKAHEAD=1 python tools/bench_algo.py getrf_1d -N 32768 --nb 512 --runs 2 || exit 1
step getrf64k 300 python tools/bench_algo.py getrf_1d -N 65536 --nb 512 --runs 1 || exit 1
step getrf64k_la_bw32 300 env DPLASMA_LU_BW=32 DPLASMA_LU_LOOKAHEAD=1 python tools/bench_algo.py getrf_1d -N 65536 --nb 512 --runs 1 || exit 1
step luqr32k 300 python tools/gpu/luqr_syncdebug.py 32768 256 || exit 1
step luqr32k_bw32 300 env DPLASMA_LU_BW=32 python tools/gpu/luqr_syncdebug.py 32768 256 || exit 1
step hqr32k_a4 200 python tools/bench_algo.py geqrf -N 32768 --nb 256 --ib 32 --runs 2 --tree hqr --qr-llvl 1 --qr-hlvl 0 --qr-a 4 || exit 1
step dist_rehearsal 300 env DPLASMA_DIST_BACKEND=gloo python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/gpu/lu_dist_rehearsal.py 16384 512 || exit 1
exit 0
