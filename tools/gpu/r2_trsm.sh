#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_potrf_tile_gpu.py tests/test_gpu_kernels.py -x -q -k "potrf or trsm or tile" \
    --timeout 120 --timeout-method thread > gpurun_out/potrf_tile_tests.log 2>&1
rc=$?; tail -4 gpurun_out/potrf_tile_tests.log; echo "tile tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/gpu/trsm_panel_bench.py 15 63 127 > gpurun_out/trsm_panel.log 2>&1
rc=$?; cat gpurun_out/trsm_panel.log; [ $rc -ne 0 ] && exit $rc
for N in 16384 32768; do
  timeout -k 10 200 python bench.py -N $N --steps 3 --warmup 1 > gpurun_out/bench_$N.log 2>&1
  rc=$?; tail -2 gpurun_out/bench_$N.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
done
exit 0
