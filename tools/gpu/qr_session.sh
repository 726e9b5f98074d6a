#!/bin/bash
# QR GPU session: numerics tests then a few timings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests/test_qr.py -m gpu -x -q > gpurun_out/qr_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/qr_gpu.log; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/bench_algo.py geqrf -N ${QR_N:-8192} --nb 256 --ib 32 > gpurun_out/qr_bench.log 2>&1
rc=$?; cat gpurun_out/qr_bench.log; echo "bench rc=$rc"
exit $rc
