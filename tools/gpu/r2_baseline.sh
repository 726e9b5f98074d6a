#!/bin/bash
# Round-2 baseline session on one MI355X: GPU test suite, the driver's exact bench command (with the
# default-on residual check), then a rocprofv3 kernel-stats profile of one 32k factorisation.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -8 gpurun_out/gpu_tests.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARM:-5} > gpurun_out/bench_driver.log 2>&1
rc=$?; tail -4 gpurun_out/bench_driver.log; echo "bench rc=$rc"
[ $rc -ne 0 ] && exit $rc
[ -n "$NOPROF" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof -o potrf32k -- \
    python3 $R/bench.py -N 32768 --steps 1 --warmup 1 --no-check > $R/gpurun_out/prof.log 2>&1
rc=$?; tail -3 $R/gpurun_out/prof.log; exit $rc
