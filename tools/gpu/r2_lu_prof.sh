#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp
DPLASMA_LU_LOOKAHEAD=${LA:-1} timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_lu -o lu32k -- \
    python3 $R/tools/bench_algo.py getrf_1d -N 32768 --nb 512 --runs 1 > $R/gpurun_out/prof_lu.log 2>&1
rc=$?; tail -2 $R/gpurun_out/prof_lu.log; exit $rc
