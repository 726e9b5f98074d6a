#!/bin/bash
# r5 batch 46: DGETRF 64k kernel split with the tagged pivot exchange (compare profiles/r4_getrf64k_kernel_stats.txt)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
O=$R/gpurun_out/r5b46
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o lu -- python3 $R/tools/bench_algo.py getrf_1d -N 65536 --nb 512 --runs 1 > $O/run.log 2>&1
rc=$?
echo "rc=$rc" > $O/summary.log
grep TIME $O/run.log | cut -c1-150 >> $O/summary.log
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && head -14 "$f" | cut -c1-160 >> $O/summary.log
cp "$f" $O/kernel_stats.csv 2>/dev/null
exit $rc
