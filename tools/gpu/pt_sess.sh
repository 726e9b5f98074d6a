#!/bin/bash
# tile POTRF/TRSM numerics, isolated tile timings + phase ablation, DPOTRF 32k/64k (one GPU)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 120 python -m pytest tests/test_gpu_kernels.py -q -x -k "potrf or trsm" --timeout 120 --timeout-method thread \
  > gpurun_out/pt_tests.log 2>&1 || { tail -20 gpurun_out/pt_tests.log; exit 1; }
tail -2 gpurun_out/pt_tests.log
timeout -k 10 120 python tools/gpu/potrf_tile_bench.py 256 512 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 120 python tools/gpu/potrf_tile_phases.py 2>&1 | grep -v amdgpu.ids || exit 1
for N in ${NS:-32768 65536}; do
  timeout -k 10 200 python bench.py -N $N --steps 2 --warmup 1 2>&1 | grep TIME || exit 1
done
