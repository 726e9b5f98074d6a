#!/bin/bash
# Kernel-time breakdown of the 1-GPU LU variants at 32k (rocprofv3 --kernel-trace --stats)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for op in getrf_nopiv getrf_1d; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_$op -o $op -- \
      python3 $R/tools/bench_algo.py $op -N 32768 --nb 512 --runs 1 > $R/gpurun_out/prof_$op.log 2>&1 || exit 1
  grep TIME $R/gpurun_out/prof_$op.log
done
