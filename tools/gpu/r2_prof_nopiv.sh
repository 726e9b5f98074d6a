#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_nopiv -o nopiv -- \
    python3 $R/tools/bench_algo.py getrf_nopiv -N 32768 --nb 512 --runs 1 > $R/gpurun_out/prof_nopiv.log 2>&1
rc=$?; grep TIME $R/gpurun_out/prof_nopiv.log; exit $rc
