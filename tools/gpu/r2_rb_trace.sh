#!/bin/bash
# Phase timeline of the dataflow tile kernel + rocprof kernel stats of a 32k DPOTRF.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python tools/gpu/potrf_rb_trace.py 512 > gpurun_out/rb_trace.log 2>&1
rc=$?; cat gpurun_out/rb_trace.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof32k -o potrf32k -- \
    python3 $R/bench.py -N 32768 --steps 1 --warmup 1 --no-check > $R/gpurun_out/prof32k.log 2>&1
rc=$?; tail -3 $R/gpurun_out/prof32k.log; exit $rc
