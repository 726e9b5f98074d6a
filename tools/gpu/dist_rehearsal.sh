#!/bin/bash
# Multi-rank rehearsal of the distributed GPU path on ONE GPU: ranks share the device and talk
# over gloo (GPU tensors staged through the host).  Exercises the 1x2, 2x2 and 2x4 grids of the
# bench (panel packing into G slabs, row bcast + column allgather, deferred NEXT/REST updates).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 DPLASMA_DIST_BACKEND=gloo DPLASMA_POTRF_DEFER_MIN_TILES=${MINT:-4}
N=${N:-8192}
for W in 2 4 8; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 \
      --master-port $((29500 + W)) bench.py --gpus $W -N $N --steps 1 --warmup 1 --check > gpurun_out/dist_w$W.log 2>&1
  rc=$?; grep -h "SUCCESS\|FAIL\|TIME\|Error\|error" gpurun_out/dist_w$W.log | head -5; echo "world=$W rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
