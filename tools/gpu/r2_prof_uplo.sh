#!/bin/bash
# Kernel stats of one DPOTRF 32k factorisation, lower and upper (where does upper lose 10 %?).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for U in L U; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_uplo_$U -o p -- python3 $R/bench.py -N 32768 --uplo $U --steps 1 --warmup 1 --no-check > $R/gpurun_out/prof_uplo_$U.log 2>&1 || exit 1
  f=$(find $R/gpurun_out/prof_uplo_$U -name "*kernel_stats.csv" | head -1)
  echo "== $U"; cut -d, -f1-4 "$f" | sed 's/(.*"//' | head -8
done
