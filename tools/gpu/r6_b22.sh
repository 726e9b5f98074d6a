#!/bin/bash
# r6 batch 22: DTR 16k trace with the POTRF phase stamps, then the priority-resolution sweep (r6_b21)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
timeout -k 10 200 python -u tools/gpu/dtr_trace_run.py 16384 gpurun_out/dtr16k_ph.npz > gpurun_out/dtr16k_ph.log 2>&1 || { tail -20 gpurun_out/dtr16k_ph.log; exit 1; }
grep -A40 "^POTRF(0)" gpurun_out/dtr16k_ph.log
bash tools/gpu/r6_b21.sh
