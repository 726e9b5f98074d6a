#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python tools/gpu/trsm_panel_bench.py 15 63 127 > gpurun_out/trsm_panel.log 2>&1
rc=$?; cat gpurun_out/trsm_panel.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof32k -o potrf32k -- \
    python3 $R/bench.py -N 32768 --steps 1 --warmup 1 --no-check > $R/gpurun_out/prof32k.log 2>&1
rc=$?; tail -2 $R/gpurun_out/prof32k.log; exit $rc
