#!/bin/bash
# diagonal-tile kernels in isolation, then DPOTRF with each tile kernel at per-GPU sizes that
# stand in for the 2/4/8-GPU shares of N=64k (one GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -m pytest tests/test_gpu_kernels.py -q -x -k "potrf" --timeout 120 --timeout-method thread \
  > gpurun_out/pt_tests.log 2>&1 || { tail -20 gpurun_out/pt_tests.log; exit 1; }
tail -2 gpurun_out/pt_tests.log
timeout -k 10 120 python tools/gpu/potrf_tile_bench.py 256 512 1024 2>&1 | grep -v amdgpu.ids || exit 1
for N in ${NS:-16384 32768}; do
  for K in single blocked; do
    DPLASMA_POTRF_TILE=$K timeout -k 10 200 python bench.py -N $N --steps 2 --warmup 1 2>&1 | grep TIME | sed "s/^/$K /" || exit 1
  done
done
