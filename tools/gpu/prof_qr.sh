#!/bin/bash
# rocprofv3 kernel-trace stats of one dgeqrf run (flat tree by default).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_qr -o qr -- python3 $R/tools/bench_algo.py geqrf -N ${QR_N:-16384} --nb 256 --ib 32 --runs 1 ${QR_ARGS} > $R/gpurun_out/prof_qr.log 2>&1
rc=$?; tail -3 $R/gpurun_out/prof_qr.log
f=$(find $R/gpurun_out/prof_qr -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -12 "$f"
exit $rc
