#!/bin/bash
# Diagonal-tile Cholesky: LDS-broadcast vs readlane elimination of the 32x32 blocks (DPLASMA_RB_CHOL).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
DPLASMA_RB_CHOL=lds timeout -k 10 300 python -u -m pytest tests/test_potrf_tile_gpu.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "potrf or chol" > gpurun_out/b13_tests.log 2>&1
rc=$?; tail -1 gpurun_out/b13_tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
for K in lane lds; do
  DPLASMA_RB_CHOL=$K timeout -k 10 120 python tools/gpu/potrf_rb_trace.py 512 16 > gpurun_out/b13_trace_$K.log 2>&1 || exit 1
  echo "$K: $(grep -E '^---' gpurun_out/b13_trace_$K.log | tr '\n' ' ')"
done
for N in 16384 32768 65536; do for K in lane lds; do
  DPLASMA_RB_CHOL=$K timeout -k 10 200 python tools/bench_algo.py potrf -N $N --nb 512 --runs 3 > gpurun_out/b13_potrf_${N}_$K.log 2>&1 || exit 1
  echo "N=$N $K: $(grep TIME gpurun_out/b13_potrf_${N}_$K.log | tail -1 | cut -c1-130)"
done; done
exit 0
