#!/bin/bash
# bench with check at 16k, full bench, then a rocprofv3 kernel-trace profile at 32k.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python bench.py -N 16384 --steps 2 --warmup 1 --check > gpurun_out/bench_16k.log 2>&1
rc=$?; cat gpurun_out/bench_16k.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_full.log 2>&1
rc=$?; cat gpurun_out/bench_full.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof -o potrf32k -- python3 $R/bench.py -N 32768 --steps 1 --warmup 0 > $R/gpurun_out/prof.log 2>&1
rc=$?; tail -5 $R/gpurun_out/prof.log; exit $rc
