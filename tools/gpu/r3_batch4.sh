#!/bin/bash
# LU dist rehearsal under sync-debug, hybrid LU-QR after the device panel change, RCCL same-GPU probe,
# kernel statistics of one 64k DPOTRF step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_lu_qr.py tests/test_gpu_lu_dist.py -m gpu -x -q --timeout 180 \
    --timeout-method thread > gpurun_out/b4_tests.log 2>&1
rc=$?; tail -2 gpurun_out/b4_tests.log; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
DPLASMA_DIST_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29613 tools/gpu/lu_dist_rehearsal.py 8192 512 2 > gpurun_out/b4_lud.log 2>&1
rc=$?; grep -h "^rank\|Error" gpurun_out/b4_lud.log | head -4; echo "lu dist sync-debug rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -m dplasma_amd.testing dgetrf_qrf -N 16384 -t 512 -x > gpurun_out/b4_luqr.log 2>&1
rc=$?; grep -E "TIME|SUCC|FAIL|Error" gpurun_out/b4_luqr.log | head -5; echo "getrf_qrf rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29661 tools/gpu/rccl_same_gpu_probe.py > gpurun_out/b4_rccl_probe.log 2>&1
echo "rccl probe rc=$?"; grep -h "RCCL_SAME_GPU\|rror" gpurun_out/b4_rccl_probe.log | head -6
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/b4_prof -o potrf -- python bench.py --steps 1 --warmup 1 \
    --no-check > gpurun_out/b4_potrf_prof.log 2>&1
echo "potrf prof rc=$?"; grep TIME gpurun_out/b4_potrf_prof.log | head -2
exit 0
