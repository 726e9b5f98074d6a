#!/bin/bash
# QR GPU tests (single rank) + P x Q stacked-domain HQR rehearsal on one GPU (gloo ranks).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_qr.py -x -q -m gpu --timeout 150 --timeout-method thread \
    > gpurun_out/qr_gpu_tests.log 2>&1 || { tail -20 gpurun_out/qr_gpu_tests.log; exit 1; }
tail -2 gpurun_out/qr_gpu_tests.log
export DPLASMA_DIST_BACKEND=gloo
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29611 tools/gpu/hqr_dist_rehearsal.py 4096 256 2 > gpurun_out/hqr_2x1.log 2>&1 \
    || { tail -30 gpurun_out/hqr_2x1.log; exit 1; }
grep hqr gpurun_out/hqr_2x1.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29612 tools/gpu/hqr_dist_rehearsal.py 4096 256 2 > gpurun_out/hqr_2x2.log 2>&1 \
    || { tail -30 gpurun_out/hqr_2x2.log; exit 1; }
grep hqr gpurun_out/hqr_2x2.log
