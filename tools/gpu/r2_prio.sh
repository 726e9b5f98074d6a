#!/bin/bash
# Wave-priority experiment on the POTRF critical-path kernels: tile tests, phase trace alone and
# beside a GEMM, isolated/beside timings, then 16k / 32k / 64k.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_potrf_tile_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/prio_tile_tests.log 2>&1 || { tail -20 gpurun_out/prio_tile_tests.log; exit 1; }
tail -1 gpurun_out/prio_tile_tests.log
timeout -k 10 120 python tools/gpu/potrf_rb_trace.py 512 > gpurun_out/prio_rb_trace.log 2>&1 || exit $?
grep -E "WG start|^ 0 |^ 7 |^14 " gpurun_out/prio_rb_trace.log
timeout -k 10 200 python tools/gpu/potrf_tile_bench.py 512 > gpurun_out/prio_tile_bench.log 2>&1 || exit $?
grep " rb " gpurun_out/prio_tile_bench.log
for N in 16384 32768 65536; do
  timeout -k 10 200 python bench.py -N $N --steps 3 --warmup 1 --no-check 2>&1 | grep TIME || exit 1
done
