#!/bin/bash
# LU block kernel A/B (register vs LDS, look-ahead on/off), hybrid LU-QR, HQR 2x4 rank replay,
# distributed LU panel with sync-debug (no host sync inside a panel) + kernel trace, RCCL same-GPU probe.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m dplasma_amd.testing dgetrf_qrf -N 16384 -t 512 -x > gpurun_out/b3_luqr.log 2>&1
rc=$?; grep -E "TIME|SUCC|FAIL|Error" gpurun_out/b3_luqr.log | head -5; echo "getrf_qrf rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/replay_hqr.py -N 65536 --nb 256 --grid 2x4 --ranks all --steps 1 --bw 65 --lat 10 \
    > gpurun_out/b3_replay_hqr.log 2>&1
rc=$?; tail -9 gpurun_out/b3_replay_hqr.log | cut -c1-400; echo "replay hqr rc=$rc"
[ $rc -ne 0 ] && exit $rc
export DPLASMA_DIST_BACKEND=gloo
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29613 tools/gpu/lu_dist_rehearsal.py 8192 512 2 > gpurun_out/b3_lud.log 2>&1
rc=$?; grep -h "^rank" gpurun_out/b3_lud.log; echo "lu dist sync-debug rc=$rc"
[ $rc -ne 0 ] && exit $rc
unset DPLASMA_DIST_BACKEND
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29661 tools/gpu/rccl_same_gpu_probe.py > gpurun_out/b3_rccl_probe.log 2>&1
echo "rccl probe rc=$?"; grep -h "RCCL_SAME_GPU" gpurun_out/b3_rccl_probe.log | head -4
exit 0
