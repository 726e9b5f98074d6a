#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r4b2
export PYTHONUNBUFFERED=1
timeout -k 10 240 python tools/gpu/prio_probe.py 96 2 0 512 768 1024 2048 > gpurun_out/r4b2/prio_96.log 2>&1
rc=$?; cat gpurun_out/r4b2/prio_96.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python tools/gpu/prio_probe.py 128 4 0 512 1024 > gpurun_out/r4b2/prio_128.log 2>&1
rc=$?; cat gpurun_out/r4b2/prio_128.log; exit $rc
