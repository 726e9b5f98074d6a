#!/bin/bash
# Full GPU test suite (one process, per-test timeout), then the driver's bench command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread \
    > gpurun_out/gpu_suite.log 2>&1
rc=$?; tail -6 gpurun_out/gpu_suite.log; echo "suite rc=$rc"
[ $rc -ne 0 ] && exit $rc
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1
rc=$?; tail -2 gpurun_out/bench_driver.log | cut -c1-700; exit $rc
