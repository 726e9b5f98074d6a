#!/bin/bash
# New diagonal-tile kernel: numerics tests (incl. under load), isolated/beside-GEMM timings, then
# the driver bench with check.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_potrf_tile_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/potrf_tile_tests.log 2>&1
rc=$?; tail -15 gpurun_out/potrf_tile_tests.log; echo "tile tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/gpu/potrf_tile_bench.py 256 512 > gpurun_out/potrf_tile_bench.log 2>&1
rc=$?; cat gpurun_out/potrf_tile_bench.log; [ $rc -ne 0 ] && exit $rc
for N in 16384 32768; do
  timeout -k 10 200 python bench.py -N $N --steps 3 --warmup 1 > gpurun_out/bench_$N.log 2>&1
  rc=$?; tail -2 gpurun_out/bench_$N.log; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 500 python bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARM:-5} > gpurun_out/bench_driver.log 2>&1
rc=$?; tail -3 gpurun_out/bench_driver.log; exit $rc
