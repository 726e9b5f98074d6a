#!/bin/bash
# Diagonal-tile kernel + panel TRSM: numerics tests (incl. under load), POTRF GPU tests, phase
# trace, isolated/beside-GEMM timings, then 16k / 32k and the driver bench with check.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_potrf_tile_gpu.py tests/test_gpu_kernels.py -x -q -k "potrf or trsm or tile" \
    --timeout 120 --timeout-method thread > gpurun_out/potrf_tile_tests.log 2>&1
rc=$?; tail -15 gpurun_out/potrf_tile_tests.log; echo "tile tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/gpu/potrf_rb_trace.py 512 > gpurun_out/rb_trace.log 2>&1
rc=$?; head -22 gpurun_out/rb_trace.log; [ $rc -ne 0 ] && exit $rc
[ -n "$TILEBENCH" ] && { timeout -k 10 200 python tools/gpu/potrf_tile_bench.py 512 > gpurun_out/potrf_tile_bench.log 2>&1 || exit $?; cat gpurun_out/potrf_tile_bench.log; }
for N in 16384 32768; do
  timeout -k 10 200 python bench.py -N $N --steps 3 --warmup 1 > gpurun_out/bench_$N.log 2>&1
  rc=$?; tail -2 gpurun_out/bench_$N.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 500 python bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARM:-5} > gpurun_out/bench_driver.log 2>&1
rc=$?; tail -3 gpurun_out/bench_driver.log | cut -c1-600; exit $rc
