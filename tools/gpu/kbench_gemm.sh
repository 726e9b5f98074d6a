#!/bin/bash
# GEMM-engine numerics tests + micro-benchmarks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gemm_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/kbench.py ${KB:-gemm} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/kbench.log
