#!/bin/bash
# Multi-rank rehearsal of the distributed GPU path on ONE GPU: ranks share the device and talk
# over gloo (GPU tensors staged through the host).  Exercises the bench's grids (2x1, 4x1, 2x4 for
# lower; 1x2, 1x4 for upper): panel packing into G slabs, row bcast + column allgather, deferred updates.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 DPLASMA_DIST_BACKEND=gloo DPLASMA_POTRF_DEFER_MIN_TILES=${MINT:-4}
N=${N:-8192}
for WU in 2:L 4:L 8:L 2:U 4:U; do
  W=${WU%:*}; U=${WU#*:}
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 \
      --master-port $((29500 + W)) bench.py --gpus $W -N $N --uplo $U --steps 1 --warmup 1 --check \
      > gpurun_out/dist_w${W}_$U.log 2>&1
  rc=$?; grep -h "SUCCESS\|FAIL\|TIME\|Error\|error" gpurun_out/dist_w${W}_$U.log | head -5; echo "world=$W uplo=$U rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
