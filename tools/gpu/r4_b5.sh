#!/bin/bash
# r4 batch 5: DTR per-task timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r4b5
export PYTHONUNBUFFERED=1
timeout -k 10 200 python tools/gpu/dtr_trace_run.py 8192 gpurun_out/r4b5/dtr8k.npz > gpurun_out/r4b5/dtr8k.log 2>&1
rc=$?; cat gpurun_out/r4b5/dtr8k.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/gpu/dtr_trace_run.py 32768 gpurun_out/r4b5/dtr32k.npz > gpurun_out/r4b5/dtr32k.log 2>&1
rc=$?; cat gpurun_out/r4b5/dtr32k.log; exit $rc
