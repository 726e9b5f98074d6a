#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/b7_prof -o luqr -- python tools/gpu/luqr_prof.py 8192 512 \
    > gpurun_out/b7_luqr.log 2>&1
rc=$?; grep "^run" gpurun_out/b7_luqr.log; echo "rc=$rc"
f=$(ls gpurun_out/b7_prof/*kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && head -15 "$f" | cut -c1-200
exit $rc
