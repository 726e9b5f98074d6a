#!/bin/bash
# r4 batch 34: per-kernel time of the hybrid LU-QR at N=32768 NB=256 (DEFAULT criterion), for the next round's plan
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4b34
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o luqr -- python3 tools/gpu/luqr_syncdebug.py 32768 256 > $O/luqr_prof.log 2>&1
rc=$?
echo "rc=$rc" >> $O/luqr_prof.log
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cut -c1-220 "$f" | head -25 > $O/kernel_stats_top.txt
find $O/prof -name "*.csv" ! -name "*kernel_stats.csv" -delete 2>/dev/null
find $O/prof -name "*.db" -delete 2>/dev/null
exit $rc
