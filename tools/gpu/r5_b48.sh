#!/bin/bash
# r5 batch 48: tagged LU exchange -- polling with s_sleep(1) (default) vs a tight spin (libdplasma_kernels_spin.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=gpurun_out/r5b48
mkdir -p $O
export PYTHONUNBUFFERED=1
for v in sleep spin; do
  L=""; [ $v = spin ] && L="DPLASMA_KERNELS_LIB=$R/dplasma_amd/lib/libdplasma_kernels_spin.so"
  echo "== $v" | tee -a $O/summary.log
  env $L timeout -k 10 120 python tools/gpu/lu_block_bench.py 1024 8192 65536 2>&1 | grep column | tee -a $O/summary.log || exit 1
  env $L timeout -k 10 200 python tools/bench_algo.py getrf_1d -N 32768 --nb 512 --runs 2 2>&1 | grep TIME | tail -1 | cut -c1-140 | tee -a $O/summary.log || exit 1
done
exit 0
