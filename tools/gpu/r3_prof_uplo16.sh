#!/bin/bash
# Kernel stats of DPOTRF 16k (chain-bound), lower vs upper.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for U in L U; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/pu16_$U -o p -- python3 $R/bench.py -N 16384 --uplo $U --steps 2 --warmup 1 --no-check > $R/gpurun_out/pu16_$U.log 2>&1 || exit 1
done
