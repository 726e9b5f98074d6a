#!/bin/bash
# r6 batch 2: bench.py N > 1 engine race with the POISONED checked run (ranks sharing one GPU, gloo host side),
# per-step times of every rank (DPLASMA_BENCH_STEPLOG=1) to explain the round-5 w4 anomaly (race 40 ms vs 269 ms/step)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6b2
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {
  local tag=$1
  shift
  echo "== $tag" | tee -a $O/summary.log
  env DPLASMA_DIST_BACKEND=gloo DPLASMA_BENCH_STEPLOG=1 "$@" > $O/$tag.log 2>&1
  local rc=$?
  grep -E "bench:|TIME|unavailable|failed|Error" $O/$tag.log | cut -c1-300 | tail -14 | tee -a $O/summary.log
  echo "rc=$rc" | tee -a $O/summary.log
  return $rc
}
run w2_16k DPLASMA_DTR_WG=128 timeout -k 10 300 python -m torch.distributed.run --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29523 bench.py --gpus 2 -N 16384 --steps 3 --warmup 1 || exit 1
run w4_16k DPLASMA_DTR_WG=64 timeout -k 10 300 python -m torch.distributed.run --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29525 bench.py --gpus 4 -N 16384 --steps 3 --warmup 1 || exit 1
exit 0
