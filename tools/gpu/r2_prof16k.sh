#!/bin/bash
# Kernel trace of the 16k DPOTRF (critical-path regime: the per-GPU share of 64k on 8 GPUs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/prof16k -o potrf16k -- \
    python3 $R/bench.py -N 16384 --steps 1 --warmup 1 --no-check > $R/gpurun_out/prof16k.log 2>&1
rc=$?; grep TIME $R/gpurun_out/prof16k.log; exit $rc
