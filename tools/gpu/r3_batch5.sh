#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/gpu/luqr_prof.py 32768 256 > gpurun_out/b5_luqr_prof.log 2>&1
rc=$?; grep "^run" gpurun_out/b5_luqr_prof.log; echo "rc=$rc"; exit $rc
