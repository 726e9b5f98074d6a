#!/bin/bash
# Capped tile DAGs + device pltmg GPU tests; kernel + memory-copy trace of the distributed LU panel
# rehearsal (rank 0); hybrid LU-QR and 1-GPU LU numbers; RCCL two-ranks-on-one-GPU probe.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_capped.py tests/test_aux_extra.py tests/test_potrf_ooc.py \
    tests/test_api_variants.py tests/test_lu.py tests/test_lu_qr.py tests/test_gpu_lu_dist.py -m gpu -x -v \
    --timeout 180 --timeout-method thread > gpurun_out/b2_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/b2_tests.log | tail -12; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
# rank-0 kernel + memory copy trace of the 2-rank distributed LU panel (gloo setup, IPC exchange)
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29655 WORLD_SIZE=2 DPLASMA_DIST_BACKEND=gloo
( RANK=1 LOCAL_RANK=1 timeout -k 10 200 python tools/gpu/lu_dist_rehearsal.py 8192 512 2 > gpurun_out/b2_lud_r1.log 2>&1 ) &
pid=$!
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
RANK=0 LOCAL_RANK=0 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/b2_prof -o lud \
    -- python tools/gpu/lu_dist_rehearsal.py 8192 512 2 > gpurun_out/b2_lud_r0.log 2>&1
rc0=$?; wait $pid; rc1=$?
grep -h "^rank" gpurun_out/b2_lud_r0.log gpurun_out/b2_lud_r1.log; echo "lu dist trace rc=$rc0/$rc1"
[ $rc0 -ne 0 ] && exit $rc0
unset MASTER_ADDR MASTER_PORT WORLD_SIZE DPLASMA_DIST_BACKEND
# hybrid LU-QR (reference testing_zgetrf_qrf defaults) and LU variants on one GPU
timeout -k 10 300 python -m dplasma_amd.testing dgetrf_qrf -N 16384 -t 512 -x > gpurun_out/b2_luqr.log 2>&1
rc=$?; grep -E "TIME|SUCC|FAIL|Error" gpurun_out/b2_luqr.log | head -5; echo "getrf_qrf rc=$rc"
[ $rc -ne 0 ] && exit $rc
# partial-pivoting LU: register-resident vs LDS block kernel, with and without look-ahead
for N in 32768 65536; do for K in reg lds; do for LA in 0 1; do
  DPLASMA_LU_BLOCK=$K DPLASMA_LU_LOOKAHEAD=$LA timeout -k 10 200 python tools/bench_algo.py getrf_1d -N $N --nb 512 --runs 2 \
      > gpurun_out/b2_lu_${N}_${K}_${LA}.log 2>&1 || { echo "lu $N $K $LA failed"; tail -5 gpurun_out/b2_lu_${N}_${K}_${LA}.log; exit 1; }
  echo "N=$N block=$K lookahead=$LA: $(grep TIME gpurun_out/b2_lu_${N}_${K}_${LA}.log | tail -1 | cut -c1-150)"
done; done; done
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29661 tools/gpu/rccl_same_gpu_probe.py > gpurun_out/b2_rccl_probe.log 2>&1
echo "rccl probe rc=$?"; grep -h "RCCL_SAME_GPU" gpurun_out/b2_rccl_probe.log | head -4
exit 0
