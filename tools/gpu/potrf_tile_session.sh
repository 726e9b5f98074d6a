#!/bin/bash
# Cholesky-family GPU tests, tile-POTRF micro-benchmarks (multi-workgroup vs single-workgroup
# kernel) and the 16k / 64k benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "potrf or posv or poinv or cholesky or chol or capi" --timeout 120 --timeout-method thread > gpurun_out/pt_tests.log 2>&1
rc=$?; tail -3 gpurun_out/pt_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/kbench.py potrf 2>&1 | grep -v amdgpu.ids
rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && exit $rc
DPLASMA_POTRF_MW=0 timeout -k 10 120 python tools/kbench.py potrf 2>&1 | grep -v amdgpu.ids
rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py -N 16384 --steps 2 --warmup 1 --check 2>&1 | grep -v amdgpu.ids | tail -2
rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 2 --warmup 1 2>&1 | grep -v amdgpu.ids | tail -1
