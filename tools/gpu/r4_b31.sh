#!/bin/bash
# r4 batch 31: the multi-rank GPU path of bench.py rehearsed on one GPU (2 and 4 ranks sharing it; the 8-rank case is the driver's, gloo moving the
# tiles through the host) -- plumbing only (distributed engine, grid selection, residual check), not performance.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4b31
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $O/summary.log
  timeout -k 10 $to "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -E '"metric"|Error|error|TIME' $O/$name.log | grep -v amdgpu.ids | cut -c1-400 | tail -4 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
step bench_w2 400 env DPLASMA_DIST_BACKEND=gloo $R --nproc-per-node 2 --master-port 29561 bench.py --gpus 2 --steps 1 --warmup 1 -N 16384 || exit 1
step bench_w4 400 env DPLASMA_DIST_BACKEND=gloo $R --nproc-per-node 4 --master-port 29562 bench.py --gpus 4 --steps 1 --warmup 1 -N 16384 || exit 1
exit 0
