#!/bin/bash
# Rolled diagonal-block elimination in k_potrf_rb / k_trsm_rb_prep: tile + potrf GPU tests, phase
# timeline alone / beside GEMM, tile bench, then DPOTRF lower/upper 16k/32k and the 64k headline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
out=gpurun_out/r3_rb.log; : > $out
timeout -k 10 400 python -u -m pytest tests/test_potrf_tile_gpu.py tests/test_gpu_kernels.py -x -q -m gpu --timeout 150 \
    --timeout-method thread > gpurun_out/r3_rb_tests.log 2>&1 || { tail -30 gpurun_out/r3_rb_tests.log; exit 1; }
tail -2 gpurun_out/r3_rb_tests.log >> $out
timeout -k 10 120 python tools/gpu/potrf_rb_trace.py 512 >> $out 2>&1 || { tail -20 $out; exit 1; }
timeout -k 10 200 python tools/gpu/potrf_tile_bench.py >> $out 2>&1 || { tail -20 $out; exit 1; }
for U in L U; do for N in 16384 32768; do
  timeout -k 10 200 python bench.py -N $N --uplo $U --steps 3 --warmup 1 2>&1 | grep -E "TIME|check" >> $out || { tail -20 $out; exit 1; }
done; done
timeout -k 10 300 python bench.py --steps 3 --warmup 1 2>&1 | grep -E "TIME|metric" >> $out || { tail -20 $out; exit 1; }
grep -v amdgpu.ids $out
