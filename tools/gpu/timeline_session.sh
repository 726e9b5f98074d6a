#!/bin/bash
# vendor-GEMM calibration + kernel-trace timeline of the 64k POTRF (1 warm-up-free step).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python tools/gpu/gemm_ceiling.py > gpurun_out/gemm_ceiling.log 2>&1
rc=$?; cat gpurun_out/gemm_ceiling.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/tl -o potrf64k -- python3 $R/bench.py -N 65536 --steps 1 --warmup 0 > $R/gpurun_out/tl.log 2>&1
rc=$?; tail -3 $R/gpurun_out/tl.log; exit $rc
