#!/bin/bash
# r5 batch 37: bench.py multi-rank path with the warmup engine race, rehearsed with ranks sharing one GPU (gloo)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5b37
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {
  echo "== $1" | tee -a $O/summary.log
  shift
  env DPLASMA_DIST_BACKEND=gloo "$@" > $O/run.log 2>&1
  local rc=$?
  grep -E "bench:|TIME|metric|unavailable|failed|Error" $O/run.log | cut -c1-400 | tail -6 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
run "w2 16k race" DPLASMA_DTR_WG=128 timeout -k 10 400 python -m torch.distributed.run --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29523 bench.py --gpus 2 -N 16384 --steps 2 --warmup 1 || exit 1
run "w4 16k race" DPLASMA_DTR_WG=64 timeout -k 10 400 python -m torch.distributed.run --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29525 bench.py --gpus 4 -N 16384 --steps 2 --warmup 1 || exit 1
run "w2 16k stream only" DPLASMA_BENCH_DIST_ENGINE=stream timeout -k 10 400 python -m torch.distributed.run \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29527 bench.py --gpus 2 -N 16384 --steps 2 --warmup 1 || exit 1
exit 0
