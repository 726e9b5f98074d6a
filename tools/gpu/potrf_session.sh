#!/bin/bash
# potrf GPU tests, 16k bench with check, 64k bench, and a 64k kernel-trace timeline (warm: 2nd run)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "potrf or gemm" --timeout 120 --timeout-method thread > gpurun_out/potrf_tests.log 2>&1
rc=$?; tail -3 gpurun_out/potrf_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py -N 16384 --steps 2 --warmup 1 --check > gpurun_out/bench_16k.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/bench_16k.log | tail -3; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_full.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/bench_full.log | tail -2; [ $rc -ne 0 ] && exit $rc
[ -n "$NO_TRACE" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/tl -o potrf64k -- python3 $R/bench.py -N 65536 --steps 1 --warmup 1 > $R/gpurun_out/tl.log 2>&1
rc=$?; grep TIME $R/gpurun_out/tl.log; exit $rc
