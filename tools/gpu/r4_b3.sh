#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r4b3
export PYTHONUNBUFFERED=1
echo "GPU_MAX_HW_QUEUES=$GPU_MAX_HW_QUEUES"
timeout -k 10 240 python tools/gpu/prio_probe.py 64 2 0 512 > gpurun_out/r4b3/prio_64.log 2>&1
rc=$?; cat gpurun_out/r4b3/prio_64.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/r4b3/prof -o probe -- python tools/gpu/prio_probe.py 64 2 0 > gpurun_out/r4b3/prof.log 2>&1
rc=$?; tail -3 gpurun_out/r4b3/prof.log; exit $rc
