#!/bin/bash
# zpotrf 32k: tile kernel choice (single-workgroup vs blocked MFMA sub-steps) and kernel breakdown; zgeqrf baseline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
mkdir -p gpurun_out
for T in auto blocked; do
  echo "DPLASMA_POTRF_TILE=$T"
  DPLASMA_POTRF_TILE=$T timeout -k 10 300 python tools/gpu/zgemm_bench.py 1024 32768 2>&1 | grep TIME || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_zpotrf -o zpotrf -- \
    python3 $R/tools/gpu/zgemm_bench.py 1024 16384 > $R/gpurun_out/prof_zpotrf.log 2>&1 || exit 1
cd $R
timeout -k 10 300 python tools/bench_algo.py geqrf -N 8192 --nb 256 --ib 32 --prec z --runs 1 2>&1 | grep TIME
