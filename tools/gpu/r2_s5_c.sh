#!/bin/bash
# Upper panel TRSM with LDS-staged coalesced strips: POTRF / TRSM GPU tests, PTG->DTD GPU test, then the
# lower / upper timing comparison.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "potrf or trsm or ptg" --timeout 120 \
    --timeout-method thread > gpurun_out/gpu_s5c.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_s5c.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu/r2_uplo.sh
