#!/bin/bash
# Distributed-pivoting LU panel on one GPU (2 and 4 ranks, IPC exchange), then the GPU suite + smoke + bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 DPLASMA_DIST_BACKEND=gloo
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29611 tools/gpu/lu_dist_rehearsal.py 2048 256 2 > gpurun_out/r3_lu_dist_2.log 2>&1
rc=$?; grep -h "rank\|Error\|error" gpurun_out/r3_lu_dist_2.log | tail -8; echo "lu_dist w2 rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29612 tools/gpu/lu_dist_rehearsal.py 16384 512 2 > gpurun_out/r3_lu_dist_2b.log 2>&1
rc=$?; grep -h "rank\|Error\|error" gpurun_out/r3_lu_dist_2b.log | tail -8; echo "lu_dist w2 16k rc=$rc"
[ $rc -ne 0 ] && exit $rc
unset DPLASMA_DIST_BACKEND
bash tools/gpu/r3_suite.sh
